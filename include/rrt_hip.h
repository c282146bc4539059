/*
 * rrt_hip.h — C-ABI of librrt_hip.so, the MI355X (gfx950) path-tracing backend.
 *
 * This is the drop-in boundary for the reference's GPU-backend slot:
 *   src/main.rs:58-71            `--backend cuda` -> cuda::render_in_one_weekend()
 *   src/cuda/mod.rs:337-439      imp::render(camera, &spheres, &materials) -> Result<(), String>
 *   src/gpu/mod.rs:124-301       build_in_one_weekend_scene() -> (CameraUniform, Vec<SphereGpu>, Vec<MaterialGpu>)
 *   src/render_io.rs:3-31        write_ppm_from_accum(w, h, &[f32] RGBA accum, spp)
 *
 * Plain C types only (no torch / HIP types in signatures). Every entry point returns
 * 0 on success or a negative RRT_E* code; rrt_hip_last_error() then holds the message
 * (thread-local, valid until the next call on that thread) — the Rust shim maps a
 * non-zero return to Err(rrt_hip_last_error()) exactly like cuda/mod.rs maps its
 * `map_err(|e| format!(...))` strings.
 *
 * Struct layouts are byte-identical to the reference's #[repr(C)] Pod structs, so the
 * Rust side passes `bytemuck::cast_slice` views of its existing vectors unchanged.
 */
#ifndef RRT_HIP_H
#define RRT_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* 1: book 1; 2: RrtSceneExt (motion, Perlin), kinds 5-6; 3: quads, constant-density media and
 * book-3 light lists in RrtSceneExt, kind 7, RRT_FLAG_BOOK3, rrt_build_next_week_scene /
 * rrt_build_rest_of_your_life_scene with struct outputs; 4: RrtBvhInfo.node_stride (80-B LDS /
 * 64-B global BVH2 nodes), xoshiro128+ path streams, tail-split accumulation chunks;
 * 5: exit_skip (f32 bounces never re-hit the primitive they leave), rrt_hip_render_rgb8_ex,
 * rrt_quantize_accum_books, chunk partials bounded by RRT_PARTIAL_MB (sample passes);
 * 6: RrtBvhInfo.n_unbounded (scene-enclosing media tested after the BVH walk; was _pad);
 * 7: RRT_FLAG_F64 (the books path's f64 arithmetic), rrt_hip_render_f64, rrt_render_tile_f64_async,
 * rrt_quantize_accum_books_f64; 8: RrtTile bands dealt in serpentine order (was b % n_ranks);
 * 9: rrt_accum_chunk() = 256 and the frame's chunk halved while S <= 2K down to a quarter (frames
 * over 512 samples sum in chunks of 256; was 128), rrt_testing_device_wrap, rrt_testing_recip_check
 * (test-only entry points, no drop-in counterpart); 10: tail chunks of K/4 samples (was K/8), the
 * f64 books path's sums in camera.rs:72-76's sample order with the throughput formed back to front
 * (bit-identical to the books path), rrt_testing_f64_layout; 11: frames of at most
 * rrt_accum_chunk() / 4 samples (no big chunk) keep tail chunks of K/8; rrt_testing_trig32_check. */
#define RRT_ABI_VERSION 11u

/* ---- scene ABI (== src/gpu/mod.rs:13-42) ------------------------------------------ */

/* == CameraUniform (gpu/mod.rs:15-25), 144 B.
 * params_f = [defocus_radius, image_width, image_height, samples_per_pixel]
 * params_u = [max_depth, sample_seed, n_spheres, background_mode(0 sky, 1 `background`)] */
typedef struct RrtCamera {
    float origin[4];
    float pixel00[4];
    float pixel_delta_u[4];
    float pixel_delta_v[4];
    float u[4];
    float v[4];
    float background[4];
    float params_f[4];
    uint32_t params_u[4];
} RrtCamera;

/* == SphereGpu (gpu/mod.rs:29-33), 32 B. */
typedef struct RrtSphere {
    float center_radius[4];
    uint32_t material_index;
    uint32_t _pad[3];
} RrtSphere;

/* == MaterialGpu (gpu/mod.rs:37-42), 32 B. kind 0..2 are the reference's; 3..6 extend the
 * ABI for book 2 (the_next_week/material.rs:27-53,116-135, texture.rs:39-77,111-126):
 *   3 = textured Lambertian, _pad[0] = texture index into the RrtTexture array
 *   4 = diffuse light, albedo_fuzz.xyz = emitted radiance
 *   5 = Lambertian with a solid-colour CheckerTexture: albedo_fuzz.xyz = even colour,
 *       albedo_fuzz[3] = inv_scale (1/scale), odd colour = (ref_idx, bits of _pad[0], bits of _pad[1])
 *   6 = Lambertian with a NoiseTexture: albedo_fuzz[3] = scale, _pad[0] = Perlin table index
 *       into RrtSceneExt.perlin
 *   7 = Isotropic (material.rs:137-158), albedo_fuzz.xyz = albedo: the phase function of a
 *       medium (RrtMedium); scatters into random_unit_vector() */
typedef struct RrtMaterial {
    float albedo_fuzz[4];
    uint32_t kind;
    float ref_idx;
    uint32_t _pad[2];
} RrtMaterial;

enum {
    RRT_MAT_LAMBERTIAN = 0,
    RRT_MAT_METAL = 1,
    RRT_MAT_DIELECTRIC = 2,
    RRT_MAT_TEXTURED_LAMBERTIAN = 3,
    RRT_MAT_DIFFUSE_LIGHT = 4,
    RRT_MAT_CHECKER_LAMBERTIAN = 5,
    RRT_MAT_NOISE_LAMBERTIAN = 6,
    RRT_MAT_ISOTROPIC = 7
};

/* == Perlin (the_next_week/perlin.rs:4-22): 256 unit random vectors and the three
 * permutations of 0..255. 4 KB. The reference draws them from the thread-local entropy RNG;
 * rrt_build_next_week_scene draws them from a seeded stream (parity unpinned). */
typedef struct RrtPerlin {
    float randvec[256][4]; /* xyz, w unused */
    uint16_t perm_x[256];
    uint16_t perm_y[256];
    uint16_t perm_z[256];
    uint16_t _pad[256];
} RrtPerlin;

/* == Quad (the_next_week/quad.rs:9-41), 64 B: corner q, edge vectors u, v (xyz; w unused) and
 * its material. Instanced quads (RotateY / Translate, hittable.rs:65-170) are passed already
 * transformed to world space (rrt_build_next_week_scene bakes make_box + RotateY + Translate). */
typedef struct RrtQuad {
    float q[4];
    float u[4];
    float v[4];
    uint32_t material_index;
    uint32_t _pad[3];
} RrtQuad;

/* == ConstantMedium (the_next_week/constant_medium.rs), 48 B: a volume of constant density inside a
 * boundary — a sphere (boundary_kind 0: center xyz, radius in `sphere`) or a set of quads
 * (boundary_kind 1: RrtSceneExt.boundary_quads[first .. first + count), e.g. a baked make_box).
 * The boundary is not a surface of the scene (add it separately if it is one). material_index
 * names the phase function (RRT_MAT_ISOTROPIC). Free-flight draw: the reference takes
 * `random_double()` from its entropy stream inside hit(), so its stream position depends on the
 * BVH walk; here the draw is u = splitmix64(path_rng ^ (bounce << 32) ^ medium) >> 40 (path_rng:
 * the first 64 bits of the path's xoshiro128+ state at the segment start; 24 bits,
 * times 2^-24) — one independent uniform per (path, segment, medium), the same whichever order a
 * BVH tests the primitives in. hit_distance = (-1/density) * ln(u) in f32 (a Cephes logf). */
typedef struct RrtMedium {
    float sphere[4];
    uint32_t boundary_kind;
    uint32_t first;
    uint32_t count;
    uint32_t material_index;
    float density;
    uint32_t _pad[3];
} RrtMedium;

enum { RRT_BOUNDARY_SPHERE = 0, RRT_BOUNDARY_QUADS = 1 };

/* == a book-3 light-list entry (the_rest_of_your_life/mod.rs `lights`, sampled by HittablePdf,
 * pdf.rs:58-78): a Quad (kind 0: corner q = a.xyz, edges u, v; quad.rs:93-107 pdf_value /
 * random) or a Sphere (kind 1: center a.xyz, radius a[3]; sphere.rs:55-66, 102-122). 64 B.
 * Sampling targets only: not surfaces of the scene (add those separately). */
typedef struct RrtLight {
    uint32_t kind;
    uint32_t _pad[3];
    float a[4];
    float u[4];
    float v[4];
} RrtLight;

enum { RRT_LIGHT_QUAD = 0, RRT_LIGHT_SPHERE = 1 };

/* Book-2 scene data beyond the flat sphere/material ABI. NULL = none.
 * sphere_motion: n_spheres x 4 floats, (center2 - center1).xyz of Sphere::new_moving
 * (the_next_week/sphere.rs:24-40; the sphere's center at ray time t is center1 + t*motion;
 * zero = static). Requires RRT_FLAG_RAY_TIME (rays carry the camera's time draw).
 * quads: n_quads quads (materials: Lambertian, checker, noise, metal, dielectric or light;
 * not image-textured). media: n_media constant-density volumes; boundary_quads: the quads their
 * quad boundaries index (material_index unused). Primitive order for rrt_build_bvh_ex:
 * spheres, then quads (n_spheres + j), then media (n_spheres + n_quads + m). */
typedef struct RrtSceneExt {
    const float *sphere_motion;
    const RrtPerlin *perlin;
    uint32_t n_perlin;
    uint32_t n_quads;
    const RrtQuad *quads;
    const RrtMedium *media;
    uint32_t n_media;
    uint32_t n_boundary_quads;
    const RrtQuad *boundary_quads;
    const RrtLight *lights; /* book 3 (RRT_FLAG_BOOK3): the MIS light list */
    uint32_t n_lights;
    uint32_t _pad;
} RrtSceneExt;

/* Image texture, RGB8 row-major (rtw_image.rs:57-67 `to_rgb8().into_raw()`). Borrowed. */
typedef struct RrtTexture {
    const uint8_t *rgb8;
    int32_t width;
    int32_t height;
} RrtTexture;

/* == config::RenderOverrides (config.rs:1-14): has_* = Some(..). */
typedef struct RrtOverrides {
    int32_t has_aspect_ratio;   double aspect_ratio;
    int32_t has_image_width;    int32_t image_width;
    int32_t has_samples_per_pixel; int32_t samples_per_pixel;
    int32_t has_max_depth;      int32_t max_depth;
    int32_t has_vfov;           double vfov;
    int32_t has_lookfrom;       double lookfrom[3];
    int32_t has_lookat;         double lookat[3];
    int32_t has_vup;            double vup[3];
    int32_t has_defocus_angle;  double defocus_angle;
    int32_t has_focus_dist;     double focus_dist;
    int32_t has_background;     double background[3];
} RrtOverrides;

/* ---- flags ------------------------------------------------------------------------ */
/* Book-2 camera: each camera ray draws a `time` sample after the jitter/disk draws
 * (the_next_week/camera.rs:160). Required for bit-parity with the book-2 oracle. */
#define RRT_FLAG_RAY_TIME 0x1u
/* Suppress the stderr progress lines (cuda/mod.rs:426-431 style). */
#define RRT_FLAG_QUIET 0x2u
/* Book-3 integrator (the_rest_of_your_life/camera.rs:96-254): stratified camera samples
 * (samples_per_pixel must be a square, sqrt_spp^2; sample s = s_j * sqrt_spp + s_i), one-sided
 * DiffuseLight, Lambertian / Isotropic scatter by the mixture pdf 0.5 * lights + 0.5 * material
 * (cosine / sphere pdf) over RrtSceneExt.lights, Russian roulette folded into the weight.
 * Requires RRT_FLAG_RAY_TIME (the book-3 camera draws a time per ray). */
#define RRT_FLAG_BOOK3 0x4u
/* The books path's own arithmetic (ABI v7): the kernel computes in f64, in the reference CPU path's
 * operation order (vec3.rs, sphere.rs:24-51, material.rs, camera.rs:152-209; no FP contraction),
 * on the same per-path random stream as the f32 kernel, and sums in f64 — so every path takes the
 * books path's decisions and the sums match it to a few f64 ulps (the north star's check "against
 * the repo's own CPU books path"). Book-1 scenes: material kinds 0-4, sky or background, no
 * RrtSceneExt data, not RRT_FLAG_BOOK3 (RRT_E_INVALID otherwise). Float entries return the f64 sums
 * rounded to f32; rrt_hip_render_f64 / rrt_render_tile_f64_async return them unrounded. */
#define RRT_FLAG_F64 0x8u

/* ---- error codes ------------------------------------------------------------------ */
#define RRT_OK 0
#define RRT_E_INVALID (-1)
#define RRT_E_HIP (-2)
#define RRT_E_NOMEM (-3)
#define RRT_E_NODEV (-4)
#define RRT_E_IO (-5)

/* ---- one-shot drop-in entry (replaces cuda::imp::render, cuda/mod.rs:342-439) ----------
 * Renders total_spp samples per pixel of the scene on n_gpus devices (row-interleaved
 * bands, one host thread per device), writes RGBA float accum into caller-owned
 * accum_out[W*H*4] (W,H = params_f[1], params_f[2]); accum_out[4i+3] = sample count.
 * total_spp == 0 means params_f[3] (cuda/mod.rs:384). BVH is built inside. */
int32_t rrt_hip_render(const RrtCamera *cam,
                       const RrtSphere *spheres, uint32_t n_spheres,
                       const RrtMaterial *materials, uint32_t n_materials,
                       const RrtTexture *textures, uint32_t n_textures,
                       uint32_t total_spp, uint32_t n_gpus, uint32_t flags,
                       float *accum_out);

/* rrt_hip_render with book-2 scene data (moving spheres, Perlin tables); ext may be NULL. */
int32_t rrt_hip_render_ex(const RrtCamera *cam,
                          const RrtSphere *spheres, uint32_t n_spheres,
                          const RrtMaterial *materials, uint32_t n_materials,
                          const RrtTexture *textures, uint32_t n_textures,
                          const RrtSceneExt *ext,
                          uint32_t total_spp, uint32_t n_gpus, uint32_t flags,
                          float *accum_out);

/* rrt_hip_render with RRT_FLAG_F64 implied, returning the f64 sums unrounded: accum_out[W*H*4]
 * doubles (RGB sums, [4i+3] = sample count). The books path's own arithmetic end to end (the
 * reference's CPU ray_color sums pixel_color in f64, camera.rs:73-76); quantise with
 * rrt_quantize_accum_books_f64 for the bytes camera.rs:87-94 prints. */
int32_t rrt_hip_render_f64(const RrtCamera *cam,
                           const RrtSphere *spheres, uint32_t n_spheres,
                           const RrtMaterial *materials, uint32_t n_materials,
                           const RrtTexture *textures, uint32_t n_textures,
                           uint32_t total_spp, uint32_t n_gpus, uint32_t flags,
                           double *accum_out);

/* Thread-local message for the last failing call on this thread ("" if none). */
const char *rrt_hip_last_error(void);
uint32_t rrt_hip_abi_version(void);

/* Summation order of the accum: a pixel's RGB = sum over consecutive chunks of its S samples
 * (counted from the tile's sample_begin) of each chunk's in-order sample sum, chunks added in
 * order: ((c0 + c1) + c2) + ... With K = rrt_accum_chunk() halved while S <= 2K, down to
 * rrt_accum_chunk() / 4 (ABI v9: 256 for S > 512, 128 for 256 < S <= 512, 64 below; big chunks at
 * high spp, small ones at low spp), and k = max(1, K / 4), or max(1, K / 8) for
 * S <= rrt_accum_chunk() / 4 (ABI v11; K / 8 for every S before v10): the first
 * nb = (S - 1) / K chunks hold K samples each (nb = 0 when S <= K), the remaining S - nb*K
 * samples form chunks of k (the last one possibly shorter) — small units at the end of the
 * work queue keep the persistent grid's tail short. Needed to reproduce it bit for bit.
 * The chunk partial sums live in a device buffer of at most RRT_PARTIAL_MB MiB (env, default
 * 2048); a render with more chunks than fit runs as consecutive sample passes of whole chunks,
 * each continuing the same fold, so the bits do not depend on the budget.
 * The f64 books path (RRT_FLAG_F64) sums each pixel's samples in sample order instead, as
 * camera.rs:72-76 does: ((s0 + s1) + s2) + ... from 0. */
uint32_t rrt_accum_chunk(void);

/* ---- device-resident API (bench / multi-rank hosts) --------------------------------- */
typedef struct RrtScene RrtScene;

/* A tile = the rows this rank owns (row bands of `band_rows`, dealt in serpentine order: band b
 * lies in period p = b / n_ranks at slot s = b % n_ranks and belongs to rank s when p is even,
 * n_ranks - 1 - s when p is odd) crossed with the sample range [sample_begin, sample_end). The
 * tile's rows are its bands in image order. */
typedef struct RrtTile {
    uint32_t band_rows;
    uint32_t rank;
    uint32_t n_ranks;
    uint32_t sample_begin;
    uint32_t sample_end;
} RrtTile;

/* Counters accumulated by every render launch on the scene since the last reset.
 * rays = closest-hit queries (camera + scattered: one world.hit, camera.rs:187).
 * node_visits / sphere_tests are only filled by rrt_scene_count_work (instrumented). */
typedef struct RrtCounters {
    uint64_t rays;
    uint64_t paths;
    uint64_t node_visits;
    uint64_t box_tests;
    uint64_t sphere_tests;
} RrtCounters;

/* Uploads the scene to `device`, builds the BVH (SAH, bvh.rs:21-156 criterion) on the host. */
int32_t rrt_scene_create(const RrtCamera *cam,
                         const RrtSphere *spheres, uint32_t n_spheres,
                         const RrtMaterial *materials, uint32_t n_materials,
                         const RrtTexture *textures, uint32_t n_textures,
                         uint32_t flags, int32_t device, RrtScene **out);
/* rrt_scene_create with book-2 scene data; ext may be NULL. */
int32_t rrt_scene_create_ex(const RrtCamera *cam,
                            const RrtSphere *spheres, uint32_t n_spheres,
                            const RrtMaterial *materials, uint32_t n_materials,
                            const RrtTexture *textures, uint32_t n_textures,
                            const RrtSceneExt *ext,
                            uint32_t flags, int32_t device, RrtScene **out);
int32_t rrt_scene_destroy(RrtScene *scene);

/* Number of image rows `tile` owns in an image of `height` rows (its accum is rows*W float4). */
int32_t rrt_tile_rows(uint32_t height, const RrtTile *tile, uint32_t *rows_out);
/* Global image row of the tile's local row `local_row`. */
int32_t rrt_tile_row_index(uint32_t height, const RrtTile *tile, uint32_t local_row, uint32_t *row_out);

/* Enqueue the render of `tile` on `stream` (a hipStream_t, NULL = default stream).
 * d_accum: device pointer to rows*W*4 floats, OVERWRITTEN with this tile's sums
 * (RGB sums over the tile's samples, w = sample count). Asynchronous.
 * One render in flight per RrtScene: the scene owns one work-queue head and one chunk-partial
 * buffer, so renders of the same scene must be ordered on one stream (or synchronised);
 * concurrent renders on different streams need one RrtScene each. */
int32_t rrt_render_tile_async(RrtScene *scene, const RrtTile *tile, float *d_accum, void *stream);
/* The same for a scene created with RRT_FLAG_F64: d_accum = rows*W*4 doubles (f64 sums, w = count),
 * overwritten. (rrt_render_tile_async on such a scene writes the f64 sums rounded to f32.) */
int32_t rrt_render_tile_f64_async(RrtScene *scene, const RrtTile *tile, double *d_accum, void *stream);

/* Counters (synchronises the scene's device). */
int32_t rrt_scene_read_counters(RrtScene *scene, RrtCounters *out);
int32_t rrt_scene_reset_counters(RrtScene *scene);
/* Runs the instrumented kernel variant (same seed => same paths) over `tile` into a
 * scratch accum and returns node visits / box tests / sphere tests / rays / paths. */
int32_t rrt_scene_count_work(RrtScene *scene, const RrtTile *tile, RrtCounters *out);

/* BVH summary: nodes, leaves, max depth, bytes resident. */
typedef struct RrtBvhInfo {
    uint32_t n_nodes;
    uint32_t n_leaves;
    uint32_t max_depth;
    uint32_t max_leaf_size;
    uint64_t node_bytes;
    uint64_t prim_bytes;
    uint32_t width;          /* 2: binary nodes, 4: 128-B 4-wide nodes */
    uint32_t max_leaf_param; /* leaf size the builder was asked for */
    uint32_t node_stride;    /* bytes per node: 80 (BVH2 staged in LDS: sign-ordered planes), 64 (BVH2 read
                                from global memory), 128 (BVH4); layouts in DESIGN.md */
    uint32_t n_unbounded;    /* the last n_unbounded primitives of the leaf order are not in the tree: media
                                whose boundary sphere holds the whole scene, tested after the walk (ABI v6) */
} RrtBvhInfo;
int32_t rrt_scene_bvh_info(const RrtScene *scene, RrtBvhInfo *out);

/* Host-only: the BVH rrt_scene_create would build for these spheres (width / max_leaf 0 =
 * the defaults; max_leaf <= 7 for width 2, <= 15 for width 4), as the device node array (80-B or
 * 64-B BVH2 nodes — info->node_stride, the layout scene creation picks — or 128-B BVH4 nodes,
 * layouts in DESIGN.md) and the leaf-order permutation of the spheres.
 * Call with nodes_cap 0 to size (info->node_bytes). Lets a checker walk exactly the tree the
 * kernel walks. */
int32_t rrt_build_bvh(const RrtSphere *spheres, uint32_t n_spheres, uint32_t width, uint32_t max_leaf,
                      void *nodes_out, size_t nodes_cap, uint32_t *prim_order_out, RrtBvhInfo *info);
/* The same over the book-2 scene (ext may be NULL): a moving sphere's box spans both ends of its
 * motion (Aabb::from_boxes, the_next_week/sphere.rs:31-33); quads join the primitives as indices
 * n_spheres + j (prim_order_out then holds n_spheres + n_quads entries). */
int32_t rrt_build_bvh_ex(const RrtSphere *spheres, uint32_t n_spheres, const RrtSceneExt *ext, uint32_t width,
                         uint32_t max_leaf, void *nodes_out, size_t nodes_cap, uint32_t *prim_order_out,
                         RrtBvhInfo *info);

/* ---- host-side callers of the boundary ------------------------------------------------ */

/* == gpu::build_in_one_weekend_scene (gpu/mod.rs:124-301): RTOW final scene from
 * SmallRng::seed_from_u64(seed) (reference: 0x5EED_1234) with the grid a,b in
 * [-grid_half, grid_half) (reference: 11; 50 = the 10k-sphere stress config).
 * Writes up to sphere_cap spheres/materials; *n_spheres = needed count (call with
 * cap 0 to size). ov may be NULL (= RenderOverrides::none()). */
int32_t rrt_build_in_one_weekend_scene(const RrtOverrides *ov, uint64_t seed, int32_t grid_half,
                                       RrtCamera *cam, RrtSphere *spheres, RrtMaterial *materials,
                                       uint32_t sphere_cap, uint32_t *n_spheres);

/* Book-2 scenes (the_next_week/mod.rs:68-587) flattened into the ABI: 1 bouncing_spheres,
 * 2 checkered_spheres, 3 earth, 4 perlin_spheres, 5 quads, 6 simple_light, 7 cornell_box,
 * 8 cornell_smoke, 9 final_scene(800, 10000, 40), 10 final_scene(400, 250, 4) (main.rs's
 * default arm). Random draws come from SmallRng(seed) in the books' order (the reference uses
 * the entropy RNG: parity unpinned). Instanced geometry (make_box, RotateY, Translate, the
 * rotated sphere cluster of final_scene) is baked to world space. The caller sets the *_cap
 * fields and buffers (a buffer may be NULL with cap 0 to size); every n_* is set to the count
 * needed. uses_texture0 = 1 when a material samples texture 0, the earth image the caller
 * supplies. The camera carries book 2's background (bg_mode 1); render with RRT_FLAG_RAY_TIME
 * and an RrtSceneExt over these arrays. */
typedef struct RrtBookScene {
    RrtCamera camera;
    RrtSphere *spheres;
    float *sphere_motion; /* sphere_cap x 4 floats, may be NULL */
    RrtMaterial *materials;
    RrtQuad *quads;
    RrtPerlin *perlin;
    RrtMedium *media;
    RrtQuad *boundary_quads;
    RrtLight *lights;
    uint32_t sphere_cap, n_spheres;
    uint32_t material_cap, n_materials;
    uint32_t quad_cap, n_quads;
    uint32_t perlin_cap, n_perlin;
    uint32_t media_cap, n_media;
    uint32_t boundary_quad_cap, n_boundary_quads;
    uint32_t light_cap, n_lights;
    uint32_t uses_texture0;
    uint32_t flags; /* the RRT_FLAG_* the scene renders with (RAY_TIME; BOOK3 for book 3) */
} RrtBookScene;

int32_t rrt_build_next_week_scene(int32_t scene, const RrtOverrides *ov, uint64_t seed, RrtBookScene *out);

/* The book-3 scene (the_rest_of_your_life/mod.rs:69-161): the Cornell box with one rotated box
 * and a glass sphere, the light list {the light quad, the glass sphere} for MIS. The camera's
 * samples_per_pixel is rounded down to sqrt_spp^2 (Camera::initialize, camera.rs:115-117).
 * Render with out->flags (RRT_FLAG_RAY_TIME | RRT_FLAG_BOOK3) and an RrtSceneExt over the arrays
 * (lights included). */
int32_t rrt_build_rest_of_your_life_scene(const RrtOverrides *ov, uint64_t seed, RrtBookScene *out);

/* == A node of the books' object graph (the_next_week/hittable.rs:172-180 HittableObject), for
 * rrt_flatten_scene. 112 B; the payload is f64 like the books' Vec3, rounded to f32 once, after
 * the transforms. Children of a LIST / BVH node are children[first .. first + count);
 * TRANSLATE, ROTATE_Y and CONSTANT_MEDIUM take exactly one child (count 1).
 *   SPHERE          a = center1.xyz, radius; b.xyz = center2 - center1 (Sphere::new_moving; 0 = static)
 *   QUAD            a.xyz = q, b.xyz = u, c.xyz = v
 *   LIST, BVH       (no payload; a BVH node is flattened like a list: the backend builds its own tree)
 *   TRANSLATE       a.xyz = offset (hittable.rs:65-97)
 *   ROTATE_Y        a[0] = angle in degrees (hittable.rs:99-170)
 *   CONSTANT_MEDIUM a[0] = density; material = its Isotropic phase material; the child subtree is
 *                   the boundary: one sphere, or quads only (constant_medium.rs)
 * material: the RrtMaterial index of a SPHERE / QUAD / CONSTANT_MEDIUM. */
typedef struct RrtSceneNode {
    uint32_t kind;
    uint32_t material;
    uint32_t first;
    uint32_t count;
    double a[4];
    double b[4];
    double c[4];
} RrtSceneNode;

enum {
    RRT_NODE_SPHERE = 0,
    RRT_NODE_QUAD = 1,
    RRT_NODE_LIST = 2,
    RRT_NODE_BVH = 3,
    RRT_NODE_TRANSLATE = 4,
    RRT_NODE_ROTATE_Y = 5,
    RRT_NODE_CONSTANT_MEDIUM = 6
};

/* Flatten the object graph under `root` into the ABI's flat arrays: spheres with
 * motion rows, quads, media and their boundary quads, with every Translate / RotateY composed
 * and applied to the geometry in f64 (points rotate and translate, edge and motion vectors
 * rotate) — geometrically the reference's per-ray instance transforms, once per build instead of
 * twice per ray and instance. Graph sharing (one Arc under several parents) is flattened once
 * per path, as the reference would hit it once per path. Writes into out's sphere / motion /
 * quad / media / boundary-quad arrays under their caps (caps 0 = size only); camera, materials,
 * Perlin tables and lights are the caller's and left untouched. Errors: a cycle or depth > 64,
 * a child index out of range, a medium boundary mixing spheres and quads or holding a medium. */
int32_t rrt_flatten_scene(const RrtSceneNode *nodes, uint32_t n_nodes, const uint32_t *children,
                          uint32_t n_children, uint32_t root, RrtBookScene *out);

/* Camera::initialize (in_one_weekend/camera.rs:102-150) in f64, cast to the f32 ABI as
 * gpu/mod.rs:278-298 does. lookfrom/lookat/vup are 3-vectors. */
int32_t rrt_make_camera(double aspect_ratio, int32_t image_width, int32_t samples_per_pixel,
                        int32_t max_depth, double vfov, const double *lookfrom, const double *lookat,
                        const double *vup, double defocus_angle, double focus_dist,
                        const double *background /* NULL = sky */, uint32_t sample_seed,
                        uint32_t n_spheres, RrtCamera *cam);

/* Apply RenderOverrides to a Camera's parameters (in_one_weekend/mod.rs:23-55; book 2
 * the_next_week/mod.rs:31-65 also applies `background`). in/out by pointer. */
int32_t rrt_apply_overrides(const RrtOverrides *ov, int32_t book,
                            double *aspect_ratio, int32_t *image_width, int32_t *samples_per_pixel,
                            int32_t *max_depth, double *vfov, double *lookfrom, double *lookat,
                            double *vup, double *defocus_angle, double *focus_dist,
                            double *background, int32_t *has_background);

/* == render_io::write_ppm_from_accum (render_io.rs:3-31), byte-identical P3 text.
 * Writes to `path` ("-" = stdout). */
int32_t rrt_write_ppm_from_accum(uint32_t width, uint32_t height, const float *accum,
                                 uint32_t samples_per_pixel, const char *path);
/* Same bytes into a caller buffer; *written = bytes needed (call with cap 0 to size). */
int32_t rrt_format_ppm_from_accum(uint32_t width, uint32_t height, const float *accum,
                                  uint32_t samples_per_pixel, char *buf, size_t cap, size_t *written);
/* Quantiser only (render_io.rs:8-26): rgb8[3*W*H]. */
int32_t rrt_quantize_accum(uint32_t width, uint32_t height, const float *accum,
                           uint32_t samples_per_pixel, uint8_t *rgb8);

/* == books::in_one_weekend::color::write_color (color.rs:6-32), the books CPU path's quantiser,
 * over a float accum: per channel x = (1.0 / spp) * sum in f64 (camera.rs:107, 80), sqrt if
 * x > 0 else 0, Interval(0, 0.999).clamp, (256 * x) as i32 — so +inf gives 255 and NaN 0, where
 * render_io maps every non-finite value to 0. rgb8[3*W*H]; format P3 (the same "r g b" lines
 * camera.rs:87-94 prints) with rrt_format_pnm_from_rgb8. spp >= 1. */
int32_t rrt_quantize_accum_books(uint32_t width, uint32_t height, const float *accum,
                                 uint32_t samples_per_pixel, uint8_t *rgb8);
/* The same quantiser over f64 sums (rrt_hip_render_f64): the books path's bytes for its own f64
 * pixel_color, with no f32 rounding in between. */
int32_t rrt_quantize_accum_books_f64(uint32_t width, uint32_t height, const double *accum,
                                     uint32_t samples_per_pixel, uint8_t *rgb8);

/* ---- output step after the boundary: device quantiser, P6 ---------------
 * render_io.rs writes P3 ASCII (~25 MB at 1080p) from a float accum copied to the host
 * (16 B/pixel). These entries quantise on the device (3 B/pixel over PCIe) and format P3 or
 * binary P6 from the quantised bytes. */

/* rrt_hip_render, then the render_io quantiser on each device: rgb8_out[3*W*H] holds the
 * bytes render_io::write_ppm_from_accum would print for the float accum (identical to
 * rrt_quantize_accum of rrt_hip_render's accum_out with samples_per_pixel = total_spp). */
int32_t rrt_hip_render_rgb8(const RrtCamera *cam,
                            const RrtSphere *spheres, uint32_t n_spheres,
                            const RrtMaterial *materials, uint32_t n_materials,
                            const RrtTexture *textures, uint32_t n_textures,
                            uint32_t total_spp, uint32_t n_gpus, uint32_t flags,
                            uint8_t *rgb8_out);

/* rrt_hip_render_rgb8 with book-2/3 scene data (moving spheres, Perlin tables, quads, media,
 * light lists); ext may be NULL. Same bytes as rrt_quantize_accum of rrt_hip_render_ex's accum. */
int32_t rrt_hip_render_rgb8_ex(const RrtCamera *cam,
                               const RrtSphere *spheres, uint32_t n_spheres,
                               const RrtMaterial *materials, uint32_t n_materials,
                               const RrtTexture *textures, uint32_t n_textures,
                               const RrtSceneExt *ext,
                               uint32_t total_spp, uint32_t n_gpus, uint32_t flags,
                               uint8_t *rgb8_out);

/* Enqueue the render_io quantiser on `stream` (hipStream_t, NULL = default): d_accum =
 * n_pixels float4 (RGB sums; w ignored), d_rgb8 = n_pixels*3 bytes, scale 1/samples_per_pixel
 * in f32 as render_io.rs:10 computes it. Asynchronous; byte-identical to rrt_quantize_accum. */
int32_t rrt_quantize_accum_async(uint32_t n_pixels, const float *d_accum, uint32_t samples_per_pixel,
                                 uint8_t *d_rgb8, void *stream);

/* PNM from quantised pixels: binary = 0 -> P3 text byte-identical to
 * rrt_format_ppm_from_accum of the same image; binary = 1 -> P6 ("P6\nW H\n255\n" + rgb8).
 * *written = bytes needed (call with cap 0 to size). */
int32_t rrt_format_pnm_from_rgb8(uint32_t width, uint32_t height, const uint8_t *rgb8, int32_t binary,
                                 char *buf, size_t cap, size_t *written);
int32_t rrt_write_pnm_from_rgb8(uint32_t width, uint32_t height, const uint8_t *rgb8, int32_t binary,
                                const char *path);

/* Number of visible HIP devices (0 when no GPU). */
int32_t rrt_device_count(int32_t *count);

/* Test support, not part of the drop-in (no reference counterpart): on != 0 lets a one-shot render
 * (rrt_hip_render*, n_gpus > 1) run worker g on device g % device_count, so the multi-device path
 * runs on a one-GPU box (tests/test_gpu_multidevice.py). Off by default and at every load of the
 * library: without it n_gpus must not exceed the visible devices. Process-wide. */
void rrt_testing_device_wrap(int32_t on);

/* Test support, not part of the drop-in: forces the LDS layout in which the f64 books kernel
 * (RRT_FLAG_F64) stages a scene that fits its block — bit 0: f64-widened sphere records, bit 1: the
 * 1/r table, bit 2: the f32 pre-test records beside widened ones (with bit 0) — instead of its
 * automatic choice; -1 (the default at every load) restores it. A forced layout over the block's
 * 64 KB fails the render. Every layout renders the same bits (tests/test_gpu_books64.py).
 * Process-wide. */
void rrt_testing_f64_layout(int32_t layout);

/* Test support, not part of the drop-in: runs the f32 kernel's short reciprocal (v_rcp_f32 + one
 * fma Newton step) and short square root over every f32 bit pattern against the IEEE results;
 * mismatches (3 x u64): [0] patterns with |s| in [2^-126, 2^126), +-0, +-inf or NaN whose
 * reciprocal differs, [1] patterns with |s| < 2^126 or NaN whose clamped ray slope differs, [2]
 * patterns +-0 or |s| >= 2^-96 of either sign (negatives, infinities and NaN included) whose square
 * root differs from the IEEE one (tests/test_gpu_recip.py: all 0). */
int32_t rrt_testing_recip_check(uint64_t *mismatches);

/* Test support, not part of the drop-in (ABI v11): the largest absolute errors of the device's f32
 * acosf over every f32 in [-1, 1] (out[0]) and atanf over every f32 in [0, 1] (out[1]) against its
 * f64 acos / atan, and the bounds the f64 kernel's texel enclosures assume for them (out[2],
 * out[3]; tests/test_gpu_trig32.py: each error at most half its bound). */
int32_t rrt_testing_trig32_check(double *out);

/* Test support, not part of the drop-in (ABI v11): the f64 kernel's IEEE square root without the
 * library expansion's identity scalings (rrt_books64.hip sqrt64_big) against the library root, bit
 * for bit, on 2^28 arguments from 2^-767 to the largest finite (random and nearly-square mantissas)
 * plus +-0 and +inf: out[0] = differing results, out[1] = arguments checked
 * (tests/test_gpu_trig32.py: 0 differ). */
int32_t rrt_testing_sqrt64_check(uint64_t *out);

#ifdef __cplusplus
}
#endif
#endif /* RRT_HIP_H */
