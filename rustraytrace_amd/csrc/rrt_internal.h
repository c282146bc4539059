// rrt_internal.h — layouts shared by the host runtime (rrt_host.cpp) and the gfx950
// megakernel (rrt_kernel.hip). Not part of the public C-ABI (include/rrt_hip.h).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace rrt {

// BVH2 node, 80 B, both children's boxes stored in the parent so one node visit reads one
// record. Boxes are f32 rounded outward (and grown by the slab test's rounding bound, rrt_host.cpp
// BoxSlack) from the f64 SAH build. Each axis is stored lo, hi, lo: a ray whose 1/d_a is negative
// reads its (entry, exit) plane pair at offset 1 (hi, lo), otherwise at 0 (lo, hi), so the slab
// test takes no min/max per axis. Links: a child node index (count 0), or for a leaf its first
// primitive | count << 28 — which is also the postponed-leaf record the kernel keeps.
struct alignas(16) GNode {
    float box[2][9];    // child c, axis a: lo, hi, lo at [c][3a .. 3a+2] (f32, rounded outward)
    uint32_t link[2];   // child c: node index (internal), or first primitive | count << 28 (leaf)
};
static_assert(sizeof(GNode) == 80, "GNode must be 80 B");
// The same node in 32 B, for scenes read from global memory (beyond the LDS budget): each plane
// as an f16 rounded outward (lo down, hi up; subnormals pushed out to 0 or the smallest normal),
// lo | hi << 16 per axis, and the min/max slab test. Two 16-B loads per visit: a scene read from
// L2 spends its time in the vector memory pipeline (TA/TD busy ~90 %), and the slab test reads
// each f16 plane with v_fma_mix_f32 (exact f16 -> f32 inside the FMA), so the decode costs no
// instruction. Looser boxes only add visits (C5 +0.06 %); hits are decided by the primitive
// tests. Same-box against the 64-B f32 node (round 2's layout): C5 +7.5 %, bouncing spheres
// +4.6 %, final_scene +-0.3 %. A never-hit child is the point (65504, 65504, 65504).
//   c0[a] / c1[a] = child c's axis-a planes; link as GNode::link
struct alignas(16) GNodeH {
    uint32_t c0[3];
    uint32_t c1[3];
    uint32_t link[2];
};
static_assert(sizeof(GNodeH) == 32, "GNodeH must be 32 B");
constexpr uint32_t kLinkCountShift = 28;
constexpr uint32_t kLinkFirstMask = (1u << kLinkCountShift) - 1u;
constexpr uint32_t kMaxLeafPrims = 7;  // two leaf children's counts share one 4-bit field
constexpr uint32_t kMaxUnbounded = 4;  // media tested outside the BVH (rrt_host.cpp unbounded_media)

// BVH4 node, 128 B: the boxes of 4 children as SoA float4s (child c in component c), the
// child refs and primitive counts (0 = internal node). Collapsed from the binary SAH tree.
struct alignas(16) GNode4 {
    float4 lox, hix, loy, hiy, loz, hiz;
    int4 child;
    int4 count;
};
static_assert(sizeof(GNode4) == 128, "GNode4 must be 128 B");

// Material, SoA split into two 16-B records (kind-dependent payload).
//   a = albedo.rgb (or emitted rgb for lights), fuzz (pre-clamped to <= 1, material.rs:49)
//   b = kind, ref_idx bits, texture index, 0
struct alignas(16) GMaterial {
    float4 a;
    int4 b;
};

// Perlin tables on the device (the_next_week/perlin.rs:4-22): the 256 random unit vectors
// and the three permutations packed per index: perm_x | perm_y << 8 | perm_z << 16.
struct alignas(16) GPerlin {
    float4 randvec[256];
    uint32_t perm[256];
};

// Quad (the_next_week/quad.rs:9-41) with its derived plane: q.xyz corner, q.w = D = dot(n, q);
// u, v edges; n = unit(cross(u, v)); w = cross(u, v) / |cross(u, v)|^2 (computed in f64 on the
// host, quad.rs's `(1/x) * v` divisions, then rounded to f32). 80 B.
struct alignas(16) GQuad {
    float4 q;
    float4 u;
    float4 v;
    float4 n;
    float4 w;
};

// ConstantMedium (the_next_week/constant_medium.rs): boundary sphere (xyz, r) or quads
// [first, first + count) of KParams.quads (after the scene's own quads); neg_inv_density =
// -1/density (f64 on the host, rounded to f32). 32 B.
struct alignas(16) GMedium {
    float4 sphere;
    uint32_t kind;  // 0 sphere, 1 quads
    uint32_t first;
    uint32_t count;
    float neg_inv_density;
};

// Book-3 MIS light: sphere (center xyz, radius w) or quad (index into KParams.quads, its area
// |u x v| in f64 rounded to f32). 32 B.
struct alignas(16) GLight {
    float4 sphere;
    uint32_t kind;  // 0 quad, 1 sphere
    uint32_t quad;
    float area;
    uint32_t _pad;
};

struct GTexture {
    int32_t offset;  // byte offset into the texture pool
    int32_t width;
    int32_t height;
    int32_t pad;
};

// Everything the megakernel needs, passed by value (kernarg segment).
// n / d for 0 <= n < 2^31 and a fixed d >= 1: q = (umulhi(n, m) + n) >> s with s = ceil(log2 d),
// m = floor(2^32 (2^s - d) / d) + 1 (Granlund-Montgomery; exact, tests/test_oracle.py checks it).
// d = 0 gives {0, 0} (callers never divide by it).
struct FastDiv {
    uint32_t m, s;
};
__host__ __device__ inline FastDiv make_fastdiv(uint32_t d) {
    if (d == 0) return FastDiv{0u, 0u};
    uint32_t s = 0;
    while (s < 32 && (1ull << s) < d) ++s;
    return FastDiv{(uint32_t)((((1ull << s) - d) << 32) / d + 1ull), s};
}
__host__ __device__ inline uint32_t fast_div(uint32_t n, FastDiv f) {
    return (uint32_t)((((uint64_t)n * f.m) >> 32) + n) >> f.s;
}

// f64 sums of the books path: RGB + sample count (32 B; two 16-B stores)
struct alignas(16) D4 {
    double x, y, z, w;
};
static_assert(sizeof(D4) == 32, "D4 must be 32 B");

// A chunk partial: the RGB sums of one (chunk, pixel) — the sample count is the chunk schedule's,
// so 12 B instead of a float4's 16.
struct F3 {
    float x, y, z;
};

struct KParams {
    const void *nodes;           // GNode[] (bvh_width 2) or GNode4[] (bvh_width 4)
    const float4 *prim_cr;       // sphere center.xyz, radius — in BVH leaf order
    const GMaterial *prim_mtl;   // each primitive's material record, same order (one fetch per hit)
    const float4 *prim_motion;   // (center2 - center1).xyz per primitive, same order; null = static scene
    const GPerlin *perlin;       // Perlin tables (noise textures)
    const GQuad *quads;          // quads, then media boundary quads; a quad's leaf-order primitive record is
                                 // (q.xyz, -(1 + index)) with (normal.xyz, D) in its motion slot; a
                                 // medium's (0, 0, 0, -(1 + n_quads + index))
    const GMedium *media;
    const GLight *lights;        // book 3: the MIS light list
    const uint8_t *tex_pool;
    const GTexture *texs;
    float4 *accum;               // tile-local rows * width
    unsigned long long *counters;  // RrtCounters layout (5 x u64)

    // camera (f32, from the RrtCamera ABI; disk_u/v = u/v * defocus_radius in f32)
    float p00[3];
    float du[3];
    float dv[3];
    float center[3];
    float disk_u[3];
    float disk_v[3];
    float background[3];
    float defocus_radius;

    uint32_t max_depth;
    uint32_t seed;
    uint32_t bg_mode;
    uint32_t flags;

    uint32_t width;
    uint32_t height;
    uint32_t tile_rows;     // rows owned by this tile
    uint32_t band_rows;
    uint32_t rank;
    uint32_t n_ranks;
    uint32_t sample_begin;
    uint32_t sample_end;
    uint32_t n_work_tiles;  // 8x8 pixel tiles in this tile
    uint32_t tiles_x;

    uint32_t n_nodes;
    uint32_t n_prims;
    uint32_t n_unbounded;   // the last n_unbounded leaf-order primitives: media tested after the walk
    uint32_t n_perlin;
    uint32_t perlin_in_lds; // book-2 kernels stage the Perlin tables in LDS after the scene
    uint32_t n_quads;       // the scene's quads (boundary quads follow them)
    uint32_t n_media;
    uint32_t n_lights;
    uint32_t image_tex;     // some material samples an image texture (book-1 kernels: texture path compiled in)
    uint32_t specular;      // some material is metal or dielectric (book-1 kernels: those branches compiled in)
    uint32_t sqrt_spp;      // book 3: stratified camera samples (sqrt_spp^2 per pixel)
    float recip_sqrt_spp;   // 1/sqrt_spp in f64, rounded
    uint32_t stack_depth;   // entries needed (BVH depth + 1)
    uint32_t scene_in_lds;  // stage nodes + spheres + their materials in LDS per block
    uint32_t trav_frac;     // leave the traversal loop when <= live*trav_frac/256 lanes still traverse
    uint32_t leaf_frac;     // run the postponed-leaf loop when > live*leaf_frac/256 lanes wait on leaf tests
    uint32_t bvh_width;     // 2 or 4
    uint32_t min_waves;     // launch-bounds occupancy request (waves per SIMD)
    uint32_t global_waves;  // the same for scenes read from L2 (not staged in LDS); < 6 = no bound

    // persistent work queue: units = (pixel, sample chunk), the n_big chunks of `chunk` samples
    // of every tile first (tile-major), then the tail chunks of `chunk_small` (rrt_accum_chunk)
    uint32_t chunk;           // samples per big chunk
    uint32_t chunk_small;     // samples per tail chunk: max(1, chunk / 8)
    uint32_t n_big;           // big chunks per pixel: (S - 1) / chunk (0 when S <= chunk)
    uint32_t n_chunks;        // n_big + ceil((S - n_big * chunk) / chunk_small)
    // Sample passes: the chunks are rendered pass_chunks at a time (one launch + combine per
    // pass) so the partial buffer stays within its budget; each launch's queue holds the pass's
    // chunks [chunk_begin, chunk_begin + pass_n): its pass_big big chunks first, then its tail
    // chunks. The combine continues the same left fold over chunks, so passes never change bits.
    uint32_t pass_chunks;     // chunks per pass (host: partial budget / pixels), >= 1
    uint32_t chunk_begin;     // this launch's first chunk (set per pass by launch_render)
    uint32_t pass_n;          // this launch's chunks
    uint32_t pass_big;        // this launch's big chunks (they precede its tail chunks)
    uint32_t n_big_units;     // n_work_tiles * pass_big * 64
    uint32_t n_units;         // n_work_tiles * pass_n * 64
    uint32_t n_cus;           // compute units of the device (grid sizing)
    // Division by the queue's uniform divisors as multiply-high + add + shift (FastDiv): the
    // generic 32-bit division sequence is ~35 instructions, paid at every unit start and end.
    FastDiv fd_pass_big, fd_pass_tail, fd_tiles_x, fd_band_rows, fd_n_ranks, fd_chunk, fd_chunk_small, fd_sqrt_spp;
    uint32_t *unit_counter;   // device queue heads: kQueues counters 128 B apart (zeroed per launch)
    F3 *partial;              // [pass chunk][tile pixel] RGB partial sums when n_chunks > 1 (12 B: the
                              // combine derives the count): a chunk's pixels are contiguous, so an
                              // 8x8 tile's rows fill whole 128-B lines

    // The f64 books path (flags & kFlagF64, rrt_books64.hip); appended so the f32 kernels' field
    // offsets stay unchanged. Sums and chunk partials as D4 (RGB sums, w = count) in the same
    // layouts as accum / partial; the camera's raw u, v (defocus_disk_u = u * defocus_radius is
    // formed in f64, camera.rs:136-138).
    D4 *accum64;
    D4 *partial64;
    float cam_u[3];
    float cam_v[3];
    // 1 / r per leaf-order sphere in f64 (sphere.rs:48's (p - center) / radius is (1/r) * v,
    // vec3.rs:142-148: the same IEEE quotient, formed once on the host)
    const double *prim_inv_r64;
    uint32_t inv_r_in_lds;  // f64 kernel, scene in LDS: the 1/r table staged too (fits the block's 64 KB)
    // the camera block widened to f64 on the host, as camera.rs:136-180 forms it from the f32 ABI
    // values: pixel00, delta_u, delta_v, center, defocus_disk_u = u * radius, defocus_disk_v
    double cam64[6][3];
    // per leaf-order primitive, a dielectric's (1 / eta, r0(1 / eta), r0(eta), 0) in f64, formed on
    // the host in the reference's operations (material.rs:75-102); zeros for other materials
    const double4 *prim_diel64;
    // the f32 sphere pre-test (rrt_sphere32.h) is enabled: every sphere center and radius within
    // 2^20 (its proven domain); rec32_in_lds: the widened-record layout also stages the f32 records
    uint32_t sphere32;
    uint32_t rec32_in_lds;
    // The f64 books path's summation in camera.rs:72-76's order (seq = 1): each pixel's first
    // S - T samples are one chunk summed from 0 in the lane (written to accum64 with w = S - T), the
    // last T samples tail chunks whose per-sample radiances go to seq64 ([tail sample of the pass]
    // [tile pixel] x 3 doubles; seq_first = the pass's first tail sample, relative to sample_begin),
    // folded into accum64 in sample order after the pass (launch_render_f64_seq).
    uint32_t seq;
    uint32_t seq_first;
    double *seq64;       // [tail chunk of the pass][j < chunk_small][tile pixel] x 3: nonzero radiances packed
    uint32_t *seqmask;   // [tail chunk of the pass][tile pixel]: which of the chunk's samples they are
    // the f64 path's attenuation history ([bounce][lane slot] x 3 floats, rrt_books64.hip
    // fold_back64): max_depth x hist_lanes records; the launch keeps blocks x threads <= hist_lanes
    float *hist;
    uint32_t hist_lanes;
};

// RRT_FLAG_F64 (include/rrt_hip.h): the f64 books-arithmetic kernel (rrt_books64.hip)
constexpr uint32_t kFlagF64 = 0x8u;

// Traversal stack entries held in LDS per lane: up to 64 (BVH depth <= 63).
constexpr int kMaxStackDepth = 64;
constexpr uint32_t kQueues = 8;  // work-queue counters (blocks dealt round-robin, one per XCD)
#ifndef RRT_BLOCK
#define RRT_BLOCK 512
#endif
#ifndef RRT_WAVES
#define RRT_WAVES 6
#endif
#ifndef RRT_TILE_W
#define RRT_TILE_W 8
#endif
// work-unit tile: 64 consecutive unit ids = kTileW x kTileH pixels of one chunk
constexpr uint32_t kTileW = RRT_TILE_W, kTileH = 64u / RRT_TILE_W;
constexpr int kBlock = RRT_BLOCK;          // threads per block (4 or 8 waves)
constexpr int kWavesPerSimd = RRT_WAVES;   // launch-bounds occupancy target of the main variant
constexpr int kGlobalBlock = 256;         // book-1 kernels whose scene is read from L2: block size
#ifndef RRT_B1_GLOBAL_WAVES
#define RRT_B1_GLOBAL_WAVES 7
#endif
constexpr int kGlobalWaves = RRT_B1_GLOBAL_WAVES;  // and waves per SIMD (7: 72 VGPRs)
#ifndef RRT_B2_WAVES
#define RRT_B2_WAVES 5
#endif
#ifndef RRT_B2_BLOCK
#define RRT_B2_BLOCK 256
#endif
// Book 3 at 256 x 5 (its noise-free kernel needs ~112 VGPRs): B3 +4.8 % same-box over the
// unbounded 512-thread blocks (4 waves), +3.9 % over 256 x 4.
#ifndef RRT_B3_WAVES
#define RRT_B3_WAVES 5
#endif
constexpr int kBook2Waves = RRT_B2_WAVES;  // book-2 kernels (classes 1-3): launch bound (1 = none)
constexpr int kBook2Block = RRT_B2_BLOCK;  // and block size; book 3 and unbounded launches use kBlock
constexpr int kBook3Waves = RRT_B3_WAVES;  // book 3 (class 4): launch bound (1 = none, 512-thread blocks;
                                           // else kBook2Block-thread blocks)
// Threads per block of the render launch for a scene (rrt_kernel.hip launch_width): the host sizes
// the block's LDS (traversal stack, Perlin tables) with it. book2_class: a book-2 scene rendered by
// kernel classes 1-3 (not book 3); wide_stack: more than 65535 nodes (32-bit stack, kBlock).
inline int render_block_threads(bool book2_class, bool wide_stack, bool book3 = false) {
    if (wide_stack) return kBlock;
    if (book3) return kBook3Waves > 1 ? kBook2Block : kBlock;
    return book2_class && kBook2Waves > 1 ? kBook2Block : kBlock;
}
// Per-block LDS budget for staging the scene (BVH nodes + spheres + per-sphere materials)
// next to the stack. RTOW: 13.5 KB nodes + 486 x 48 B = 36.9 KB; + ~11 KB of stack per
// 512-thread block keeps 3 blocks (6 waves/SIMD) within the CU's 160 KB.
constexpr size_t kLdsSceneBudget = 40 * 1024;
constexpr size_t kPrimBytes = sizeof(float4) + sizeof(GMaterial);  // per primitive: sphere + material
constexpr size_t kMotionBytes = sizeof(float4);                     // + motion, scenes with moving spheres

// Launch wrappers implemented in rrt_kernel.hip.
hipError_t launch_render(const KParams &p, hipStream_t stream);
hipError_t launch_render_counting(const KParams &p, hipStream_t stream);
// render_io quantiser on the device (d_accum: n_pixels x float4; d_rgb8: n_pixels x 3 B).
hipError_t launch_quantize(const float *d_accum, uint8_t *d_rgb8, uint32_t n_pixels, float scale, hipStream_t stream);
// Test support (rrt_testing_recip_check): the kernel's recip_rn / clamped_slope against the IEEE
// quotient (and sqrt_rn_big against the IEEE sqrt) over every f32 bit pattern; d_out: 3 zeroed u64
// mismatch counters
hipError_t launch_recip_check(unsigned long long *d_out, hipStream_t stream);
// Test support (rrt_testing_trig32_check, rrt_books64.hip): the largest errors of the device's acosf
// over [-1, 1] and atanf over [0, 1] against its f64 acos / atan (d_out: 2 zeroed u64 holding f64
// bits), and the error bounds the f64 kernel's texel enclosures assume (bounds[2])
hipError_t launch_trig32_check(unsigned long long *d_out, double *bounds, hipStream_t stream);
hipError_t launch_sqrt64_check(unsigned long long *d_out, hipStream_t stream);
// Implemented in rrt_books64.hip: one sample pass of the f64 books kernel (+ its chunk combine)
// into p.accum64, and the f64 sums rounded to the f32 RGBA accum of the ABI.
hipError_t launch_render_pass_f64(const KParams &p, bool count, hipStream_t stream);
// The f64 render in sequential-sum mode (p.seq): the prefix + tail-chunk passes and the in-order
// folds of the tail samples (rrt_books64.hip).
hipError_t launch_render_f64_seq(const KParams &p, bool count, hipStream_t stream);
// LDS of the f64 kernel's block with the scene staged in its smallest form (Node112 nodes, f32
// sphere records, no 1/r table): the host stages an f64 scene only when this is <= 64 KB
size_t f64_lds_min_bytes(uint32_t n_nodes, uint32_t n_prims, uint32_t stack_depth);
hipError_t launch_accum64_to_f32(const D4 *d_accum64, float4 *d_accum, uint32_t n_pixels, hipStream_t stream);
// Test support (rrt_testing_f64_layout): force the f64 kernel's LDS layout of a staged scene (-1: auto)
void set_f64_layout(int layout);

}  // namespace rrt
