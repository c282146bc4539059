// ref_slot.cpp — TEST INFRASTRUCTURE ONLY: runs the reference's own GPU slot on the MI355X.
//
// The reference's GPU backend is a CUDA C kernel held as a string in src/cuda/mod.rs:15-335
// (`CUDA_SOURCE`, compiled at run time by NVRTC, mod.rs:366, and launched through cudarc,
// mod.rs:377-432). oracle/Makefile extracts that string from /root/reference at build time and
// compiles it unmodified with hipcc for gfx950 into oracle/_ref/ref_slot.hsaco (the HIP runtime
// header is force-included: it supplies float3/float4/uint4 and the thread indices that NVRTC
// provides implicitly). The source never enters the repository; only the code object, like any
// other built artefact, travels to the GPU box (git-ignored, not gpurun-ignored).
//
// This file is the host side of `imp::render` (cuda/mod.rs:342-439) restated in C++ (the
// reference's host is Rust/cudarc and cannot be built here): the same module load and
// function lookup ("render"), the same launch geometry (8x8 blocks over the image,
// mod.rs:393-401), passes of at most CUDA_SPP_PER_PASS = 256 samples (mod.rs:9, 384-386,
// 403-405), the per-pass seed base_seed ^ pass * 0x9E3779B9 (mod.rs:406), one zeroed float4
// accumulator that every pass adds into (mod.rs:391, kernel :330-332), a synchronize per pass
// (mod.rs:425) and one D2H copy at the end (mod.rs:434-436).
//
// Only tests/ and bench.py's reference legs load it, as a checker and a baseline — never the
// product path (rustraytrace_amd never imports oracle/).
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstring>
#include <string>

namespace {

thread_local std::string g_err;

int fail(const char *what, hipError_t e) {
    g_err = std::string(what) + ": " + hipGetErrorString(e);
    return -1;
}

#define REF_CHECK(call)                          \
    do {                                         \
        hipError_t e_ = (call);                  \
        if (e_ != hipSuccess) return fail(#call, e_); \
    } while (0)

// The kernel's `struct Camera` (mod.rs:17-27) == CameraUniform (gpu/mod.rs:13-24), 144 B.
struct alignas(16) RefCamera {
    float f[28];        // origin, pixel00, pixel_delta_u, pixel_delta_v, u, v, background
    float params_f[4];  // lens radius, width, height, samples per pixel
    uint32_t params_u[4];  // max depth, seed, -, background mode
};
static_assert(sizeof(RefCamera) == 144, "CameraUniform is 144 B");

struct Module {
    hipModule_t mod = nullptr;
    hipFunction_t fn = nullptr;
};

}  // namespace

extern "C" {

const char *ref_slot_last_error() { return g_err.c_str(); }

// Renders the scene with the reference's own kernel. camera: 144 B CameraUniform; spheres /
// materials: the 32-B SphereGpu / MaterialGpu records (gpu/mod.rs:26-42). accum_out receives
// W*H float4 (RGB sums, w = samples), exactly the buffer imp::render hands to
// write_ppm_from_accum. kernel_ms (optional) receives the summed HIP-event time of the passes.
int ref_slot_render(const char *hsaco_path, const void *camera, const void *spheres, uint32_t n_spheres,
                    const void *materials, uint32_t n_materials, float *accum_out, float *kernel_ms) {
    RefCamera cam;
    std::memcpy(&cam, camera, sizeof(cam));
    // mod.rs:381-387
    const uint32_t width = (uint32_t)cam.params_f[1];
    const uint32_t height = (uint32_t)cam.params_f[2];
    const float spp_f = cam.params_f[3] > 1.0f ? cam.params_f[3] : 1.0f;
    const uint32_t total_spp = (uint32_t)spp_f;
    const uint32_t kSppPerPass = 256u;  // CUDA_SPP_PER_PASS (mod.rs:9)
    const uint32_t spp_per_pass = kSppPerPass < total_spp ? kSppPerPass : total_spp;
    const uint32_t pass_count = (total_spp + spp_per_pass - 1) / spp_per_pass;
    const uint32_t base_seed = cam.params_u[1];
    const size_t pixels = (size_t)width * height;
    if (width == 0 || height == 0) {
        g_err = "empty image";
        return -1;
    }
    // the kernel indexes materials[sphere.material_index] unchecked (mod.rs:225): refuse a scene
    // that would read past the material table rather than launch it
    for (uint32_t i = 0; i < n_spheres; ++i) {
        uint32_t mi;
        std::memcpy(&mi, static_cast<const char *>(spheres) + 32u * i + 16u, 4);
        if (mi >= n_materials) {
            g_err = "sphere " + std::to_string(i) + " names material " + std::to_string(mi) + " of " +
                    std::to_string(n_materials);
            return -1;
        }
    }

    Module m;
    REF_CHECK(hipModuleLoad(&m.mod, hsaco_path));
    hipError_t e = hipModuleGetFunction(&m.fn, m.mod, "render");
    if (e != hipSuccess) {
        (void)hipModuleUnload(m.mod);
        return fail("hipModuleGetFunction(render)", e);
    }
    void *d_spheres = nullptr, *d_materials = nullptr, *d_accum = nullptr;
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    int rc = 0;
    auto cleanup = [&]() {
        if (ev0) (void)hipEventDestroy(ev0);
        if (ev1) (void)hipEventDestroy(ev1);
        if (d_spheres) (void)hipFree(d_spheres);
        if (d_materials) (void)hipFree(d_materials);
        if (d_accum) (void)hipFree(d_accum);
        (void)hipModuleUnload(m.mod);
    };
    do {
        // mod.rs:389-391 (a zero-length slice still gets a valid device pointer)
        if ((e = hipMalloc(&d_spheres, n_spheres ? n_spheres * 32u : 32u)) != hipSuccess) { rc = fail("hipMalloc", e); break; }
        if ((e = hipMalloc(&d_materials, n_materials ? n_materials * 32u : 32u)) != hipSuccess) { rc = fail("hipMalloc", e); break; }
        if ((e = hipMalloc(&d_accum, pixels * 16u)) != hipSuccess) { rc = fail("hipMalloc", e); break; }
        if (n_spheres && (e = hipMemcpy(d_spheres, spheres, n_spheres * 32u, hipMemcpyHostToDevice)) != hipSuccess) { rc = fail("hipMemcpy", e); break; }
        if (n_materials && (e = hipMemcpy(d_materials, materials, n_materials * 32u, hipMemcpyHostToDevice)) != hipSuccess) { rc = fail("hipMemcpy", e); break; }
        if ((e = hipMemset(d_accum, 0, pixels * 16u)) != hipSuccess) { rc = fail("hipMemset", e); break; }
        if ((e = hipEventCreate(&ev0)) != hipSuccess || (e = hipEventCreate(&ev1)) != hipSuccess) { rc = fail("hipEventCreate", e); break; }
        // mod.rs:393-401
        const uint32_t bx = 8, by = 8, gx = (width + bx - 1) / bx, gy = (height + by - 1) / by;
        float total_ms = 0.0f;
        for (uint32_t pass = 0; pass < pass_count && rc == 0; ++pass) {
            const uint32_t remaining = total_spp - pass * spp_per_pass;  // mod.rs:404-406
            uint32_t pass_spp = remaining < spp_per_pass ? remaining : spp_per_pass;
            uint32_t seed = base_seed ^ (pass * 0x9E3779B9u);
            uint32_t count = n_spheres, w = width, h = height;
            void *args[] = {&cam, &d_spheres, &count, &d_materials, &d_accum, &seed, &pass_spp, &w, &h};
            if ((e = hipEventRecord(ev0, nullptr)) != hipSuccess) { rc = fail("hipEventRecord", e); break; }
            if ((e = hipModuleLaunchKernel(m.fn, gx, gy, 1, bx, by, 1, 0, nullptr, args, nullptr)) != hipSuccess) {
                rc = fail("hipModuleLaunchKernel", e);
                break;
            }
            if ((e = hipEventRecord(ev1, nullptr)) != hipSuccess) { rc = fail("hipEventRecord", e); break; }
            if ((e = hipDeviceSynchronize()) != hipSuccess) { rc = fail("hipDeviceSynchronize", e); break; }  // mod.rs:425
            float ms = 0.0f;
            if ((e = hipEventElapsedTime(&ms, ev0, ev1)) != hipSuccess) { rc = fail("hipEventElapsedTime", e); break; }
            total_ms += ms;
        }
        if (rc != 0) break;
        if ((e = hipMemcpy(accum_out, d_accum, pixels * 16u, hipMemcpyDeviceToHost)) != hipSuccess) { rc = fail("hipMemcpy D2H", e); break; }
        if (kernel_ms) *kernel_ms = total_ms;
    } while (false);
    cleanup();
    return rc;
}

}  // extern "C"
