//! HIP/MI355X backend for RustRayTrace: the FFI shim over librrt_hip.so (include/rrt_hip.h).
//!
//! Drop-in for the reference's CUDA slot: `src/cuda/mod.rs:337-450` (`imp::render_in_one_weekend`,
//! `imp::render`, and the two feature-gated `render_in_one_weekend` wrappers at :442-450). It
//! consumes the structs `gpu::build_in_one_weekend_scene()` already produces
//! (`gpu/mod.rs:13-42, 124-301`, `#[repr(C)]` Pod, byte-identical to RrtCamera / RrtSphere /
//! RrtMaterial) and hands the RGBA accum to `render_io::write_ppm_from_accum` (`render_io.rs:3-31`),
//! so the output bytes are the ones the CUDA backend path prints.
//!
//! Install: copy this directory to `src/hip/`, add `mod hip;` and the `--backend hip` arm to
//! `src/main.rs` (integration/rust/main_rs.patch), `hip = []` under `[features]` in Cargo.toml
//! (integration/rust/Cargo.toml.fragment) and integration/rust/build.rs as the crate's build.rs.
//! tests/test_integration_rust.py checks every `extern "C"` declaration below against
//! include/rrt_hip.h (names, argument order and types, return types).

#[cfg(feature = "hip")]
mod imp {
    use crate::gpu::{build_in_one_weekend_scene, CameraUniform, MaterialGpu, SphereGpu};
    use crate::render_io::write_ppm_from_accum;
    use std::ffi::CStr;
    use std::os::raw::{c_char, c_void};

    /// == RrtTexture (include/rrt_hip.h): RGB8 row-major image, borrowed for the call.
    #[repr(C)]
    pub struct RrtTexture {
        pub rgb8: *const u8,
        pub width: i32,
        pub height: i32,
    }

    /// == RrtSceneExt (include/rrt_hip.h): book-2/3 data beyond the flat ABI. The shim passes
    /// null (book 1); the element types are opaque here because only their pointers cross.
    #[repr(C)]
    pub struct RrtSceneExt {
        pub sphere_motion: *const f32,
        pub perlin: *const c_void,
        pub n_perlin: u32,
        pub n_quads: u32,
        pub quads: *const c_void,
        pub media: *const c_void,
        pub n_media: u32,
        pub n_boundary_quads: u32,
        pub boundary_quads: *const c_void,
        pub lights: *const c_void,
        pub n_lights: u32,
        pub _pad: u32,
    }

    /// Suppress the library's own stderr progress lines (RRT_FLAG_QUIET).
    pub const RRT_FLAG_QUIET: u32 = 0x2;
    /// The books path's f64 arithmetic (RRT_FLAG_F64): checked against `--backend cpu` output.
    pub const RRT_FLAG_F64: u32 = 0x8;
    /// ABI this shim was written against (RRT_ABI_VERSION).
    pub const RRT_ABI_VERSION: u32 = 11;

    #[link(name = "rrt_hip")]
    extern "C" {
        // include/rrt_hip.h: the one-shot drop-in for cuda::imp::render (cuda/mod.rs:342-439)
        fn rrt_hip_render(cam: *const CameraUniform, spheres: *const SphereGpu, n_spheres: u32,
                          materials: *const MaterialGpu, n_materials: u32,
                          textures: *const RrtTexture, n_textures: u32,
                          total_spp: u32, n_gpus: u32, flags: u32, accum_out: *mut f32) -> i32;
        fn rrt_hip_render_ex(cam: *const CameraUniform, spheres: *const SphereGpu, n_spheres: u32,
                             materials: *const MaterialGpu, n_materials: u32,
                             textures: *const RrtTexture, n_textures: u32, ext: *const RrtSceneExt,
                             total_spp: u32, n_gpus: u32, flags: u32, accum_out: *mut f32) -> i32;
        // render + the render_io quantiser on the device (3 B/pixel to the host, same bytes)
        fn rrt_hip_render_rgb8(cam: *const CameraUniform, spheres: *const SphereGpu, n_spheres: u32,
                               materials: *const MaterialGpu, n_materials: u32,
                               textures: *const RrtTexture, n_textures: u32,
                               total_spp: u32, n_gpus: u32, flags: u32, rgb8_out: *mut u8) -> i32;
        // the books path's own f64 arithmetic and sums (RRT_FLAG_F64), and its f64 quantiser
        // (books/in_one_weekend/color.rs:6-32 write_color)
        fn rrt_hip_render_f64(cam: *const CameraUniform, spheres: *const SphereGpu, n_spheres: u32,
                              materials: *const MaterialGpu, n_materials: u32,
                              textures: *const RrtTexture, n_textures: u32,
                              total_spp: u32, n_gpus: u32, flags: u32, accum_out: *mut f64) -> i32;
        fn rrt_quantize_accum_books_f64(width: u32, height: u32, accum: *const f64, samples_per_pixel: u32,
                                        rgb8: *mut u8) -> i32;
        fn rrt_hip_last_error() -> *const c_char;
        fn rrt_hip_abi_version() -> u32;
        fn rrt_device_count(count: *mut i32) -> i32;
        // render_io.rs:3-31 byte-identical P3 (path "-" = stdout), P3/P6 from quantised bytes
        fn rrt_write_ppm_from_accum(width: u32, height: u32, accum: *const f32, samples_per_pixel: u32,
                                    path: *const c_char) -> i32;
        fn rrt_write_pnm_from_rgb8(width: u32, height: u32, rgb8: *const u8, binary: i32,
                                   path: *const c_char) -> i32;
    }

    fn last_error() -> String {
        // Thread-local message of the failing call on this thread (rrt_hip.h).
        unsafe { CStr::from_ptr(rrt_hip_last_error()) }.to_string_lossy().into_owned()
    }

    fn check(rc: i32) -> Result<(), String> {
        if rc == 0 { Ok(()) } else { Err(last_error()) }
    }

    /// Devices to render on: RRT_GPUS (default 1, capped at the visible count). Row bands are
    /// dealt over them in serpentine order inside the library (one host thread per device).
    fn gpus() -> Result<u32, String> {
        let mut visible = 0i32;
        check(unsafe { rrt_device_count(&mut visible) })?;
        if visible < 1 {
            return Err("no HIP device visible".to_string());
        }
        let want = std::env::var("RRT_GPUS").ok().and_then(|v| v.parse::<u32>().ok()).unwrap_or(1);
        Ok(want.clamp(1, visible as u32))
    }

    pub fn render_in_one_weekend() -> Result<(), String> {
        let (camera, spheres, materials) = build_in_one_weekend_scene();
        render(camera, &spheres, &materials)
    }

    /// Same contract as cuda::imp::render (cuda/mod.rs:342): render the scene and print the
    /// PPM to stdout through render_io. RRT_DEVICE_QUANTISE=1 quantises on the device instead
    /// (rrt_hip_render_rgb8 + the library's P3 writer: identical bytes, 3 B/pixel over PCIe).
    /// RRT_BOOKS_F64=1 renders with the books path's f64 arithmetic (rrt_hip_render_f64) and
    /// prints the bytes color.rs's write_color gives for the f64 sums.
    fn render(camera: CameraUniform, spheres: &[SphereGpu], materials: &[MaterialGpu]) -> Result<(), String> {
        let abi = unsafe { rrt_hip_abi_version() };
        if abi != RRT_ABI_VERSION {
            return Err(format!("librrt_hip.so ABI {abi}, shim expects {RRT_ABI_VERSION}"));
        }
        let width = camera.params_f[1] as u32;
        let height = camera.params_f[2] as u32;
        let total_spp = camera.params_f[3].max(1.0) as u32; // cuda/mod.rs:384
        let n_gpus = gpus()?;
        let pixels = width as usize * height as usize;
        if std::env::var("RRT_BOOKS_F64").map(|v| v == "1").unwrap_or(false) {
            let mut accum = vec![0.0f64; pixels * 4];
            check(unsafe {
                rrt_hip_render_f64(&camera, spheres.as_ptr(), spheres.len() as u32,
                                   materials.as_ptr(), materials.len() as u32,
                                   std::ptr::null(), 0, total_spp, n_gpus, RRT_FLAG_F64, accum.as_mut_ptr())
            })?;
            let mut rgb8 = vec![0u8; pixels * 3];
            check(unsafe { rrt_quantize_accum_books_f64(width, height, accum.as_ptr(), total_spp, rgb8.as_mut_ptr()) })?;
            let stdout = b"-\0";
            return check(unsafe {
                rrt_write_pnm_from_rgb8(width, height, rgb8.as_ptr(), 0, stdout.as_ptr() as *const c_char)
            });
        }
        if std::env::var("RRT_DEVICE_QUANTISE").map(|v| v == "1").unwrap_or(false) {
            let mut rgb8 = vec![0u8; pixels * 3];
            check(unsafe {
                rrt_hip_render_rgb8(&camera, spheres.as_ptr(), spheres.len() as u32,
                                    materials.as_ptr(), materials.len() as u32,
                                    std::ptr::null(), 0, total_spp, n_gpus, 0, rgb8.as_mut_ptr())
            })?;
            let stdout = b"-\0";
            return check(unsafe {
                rrt_write_pnm_from_rgb8(width, height, rgb8.as_ptr(), 0, stdout.as_ptr() as *const c_char)
            });
        }
        let mut accum = vec![0.0f32; pixels * 4];
        check(unsafe {
            rrt_hip_render_ex(&camera, spheres.as_ptr(), spheres.len() as u32,
                              materials.as_ptr(), materials.len() as u32,
                              std::ptr::null(), 0, std::ptr::null(),
                              total_spp, n_gpus, 0, accum.as_mut_ptr())
        })?;
        write_ppm_from_accum(width as usize, height as usize, &accum, total_spp)
    }

    #[allow(dead_code)]
    pub fn write_ppm_native(width: u32, height: u32, accum: &[f32], spp: u32) -> Result<(), String> {
        // The library's threaded render_io writer (same bytes as render_io.rs, ~30x faster at 1080p).
        let stdout = b"-\0";
        check(unsafe { rrt_write_ppm_from_accum(width, height, accum.as_ptr(), spp, stdout.as_ptr() as *const c_char) })
    }

    #[allow(dead_code)]
    pub fn render_with_flags(camera: CameraUniform, spheres: &[SphereGpu], materials: &[MaterialGpu],
                             flags: u32) -> Result<Vec<f32>, String> {
        // Float accum only (w = sample count per pixel), for callers with their own output step.
        let pixels = camera.params_f[1] as usize * camera.params_f[2] as usize;
        let mut accum = vec![0.0f32; pixels * 4];
        check(unsafe {
            rrt_hip_render(&camera, spheres.as_ptr(), spheres.len() as u32,
                           materials.as_ptr(), materials.len() as u32, std::ptr::null(), 0,
                           0, gpus()?, flags, accum.as_mut_ptr())
        })?;
        Ok(accum)
    }
}

#[cfg(feature = "hip")]
pub fn render_in_one_weekend() -> Result<(), String> {
    imp::render_in_one_weekend()
}

#[cfg(not(feature = "hip"))]
pub fn render_in_one_weekend() -> Result<(), String> {
    Err("HIP backend not enabled. Rebuild with --features hip (and RRT_HIP_LIB_DIR pointing at librrt_hip.so).".to_string())
}
