// Host-side AddressSanitizer check of libmpiv's C ABI (SURVEY.md §5 "race detection /
// sanitizers"): built against an ASan-instrumented libmpiv (host code only; GPU ASan is
// not available on this pool) and run on the CPU.  Exercises every argument-validation
// path (no device memory is touched: each call is rejected before any HIP call) and the
// host-only entry points (mpiv_render_homographies, debug options, build id).
#include <cmath>
#include <cstdio>
#include <cstring>
#include <vector>

#include "../../include/mpiv.h"

static int failures = 0;
#define EXPECT(cond)                                                     \
    do {                                                                 \
        if (!(cond)) {                                                   \
            std::printf("FAIL %s:%d %s\n", __FILE__, __LINE__, #cond);   \
            ++failures;                                                  \
        }                                                                \
    } while (0)

int main() {
    EXPECT(mpiv_abi_version() == MPIV_ABI_VERSION);
    EXPECT(std::strlen(mpiv_build_id()) == 16);
    const int64_t st5[5] = {1, 1, 1, 1, 1}, st4[4] = {1, 1, 1, 1}, st3[3] = {1, 1, 1};
    void* p = reinterpret_cast<void*>(16);
    float* f = static_cast<float*>(p);
    // null pointers / bad shapes are rejected with MPIV_ERR_ARG and a message
    EXPECT(mpiv_render(nullptr, st5, 1, 4, 4, 2, f, f, nullptr) == MPIV_ERR_ARG);
    EXPECT(mpiv_render(f, st5, 0, 4, 4, 2, f, f, nullptr) == MPIV_ERR_ARG);
    EXPECT(std::strstr(mpiv_last_error(), "bad shape") != nullptr);
    EXPECT(mpiv_pack_planes(f, st4, 4, 4, 0, f, nullptr) == MPIV_ERR_ARG);
    EXPECT(mpiv_render_packed(reinterpret_cast<float*>(8), 4, 4, 2, f, 1, f, nullptr) == MPIV_ERR_ARG);
    EXPECT(mpiv_render_packed_ct(f, 4, 4, 8, 5, 3, 0, f, 1, f, nullptr) == MPIV_ERR_ARG);
    EXPECT(mpiv_combine_ct(f, 0, 4, f, nullptr) == MPIV_ERR_ARG);
    const int64_t stb[5] = {4 * 4 * 2 * 4, 4 * 2 * 4, 2 * 4, 4, 1};  // [1,4,4,2,4] contiguous
    EXPECT(mpiv_render_backward(f, stb, 1, 4, 4, 2, f, f, nullptr, f, nullptr, 0, nullptr) == MPIV_ERR_ARG);
    EXPECT(mpiv_render_backward(f, stb, 1, 4, 4, 2, f, f, nullptr, f, reinterpret_cast<void*>(256), 0, nullptr) == MPIV_ERR_ARG);
    EXPECT(std::strstr(mpiv_last_error(), "workspace too small") != nullptr);
    EXPECT(mpiv_render_backward(f, st5, 1, 4, 4, 2, f, f, nullptr, f, reinterpret_cast<void*>(256), 0, nullptr) == MPIV_ERR_ARG);
    EXPECT(std::strstr(mpiv_last_error(), "planes contiguous per pixel") != nullptr);
    EXPECT(mpiv_render_train(f, st5, 1, 4, 4, 2, f, f, f, nullptr) == MPIV_ERR_ARG);
    EXPECT(mpiv_render_train(f, stb, 1, 4, 4, 2, f, f, nullptr, nullptr) == MPIV_ERR_ARG);
    EXPECT(mpiv_render_backward_workspace_size(0, 4, 4) == 0);
    EXPECT(mpiv_render_backward_workspace_size(64, 64, 8) > (size_t)64 * 64 * 8 * 16);
    EXPECT(mpiv_plane_sweep(f, st4, 1, 4, 4, 0, f, f, f, 2, 4, 4, f, nullptr) == MPIV_ERR_ARG);
    EXPECT(mpiv_pad_texels(f, st4, 1, 4, 4, 5, f, nullptr) == MPIV_ERR_ARG);
    EXPECT(mpiv_plane_sweep_padded_into(f, 1, 4, 4, 3, f, f, f, 2, 4, 4, f, 16, 5, nullptr) == MPIV_ERR_ARG);
    EXPECT(mpiv_inverse_warp(f, st4, 1, 4, 4, 3, f, f, nullptr, st3, 4, 4, f, nullptr) == MPIV_ERR_ARG);
    EXPECT(mpiv_grid_sample(f, st4, 0, 1, 4, 4, f, st4, 2, 2, f, st4, nullptr) == MPIV_ERR_ARG);
    EXPECT(mpiv_over_composite(nullptr, 2, 4, 4, 1, f, nullptr) == MPIV_ERR_ARG);
    EXPECT(mpiv_transform_points(f, 0, 4, f, f, nullptr) == MPIV_ERR_ARG);
    EXPECT(mpiv_normalize_homogeneous(f, 4, 0, f, nullptr) == MPIV_ERR_ARG);
    EXPECT(mpiv_pixel2cam(f, f, f, 1, 0, 1, f, nullptr) == MPIV_ERR_ARG);
    EXPECT(mpiv_cam2pixel(nullptr, f, 1, 4, f, nullptr) == MPIV_ERR_ARG);
    EXPECT(mpiv_plane_coords(f, 1, 4, f, 0, 4, f, nullptr) == MPIV_ERR_ARG);
    EXPECT(mpiv_preprocess(f, 0, f, nullptr) == MPIV_ERR_ARG);
    EXPECT(mpiv_deprocess_u8(f, 0, nullptr, nullptr) == MPIV_ERR_ARG);
    EXPECT(mpiv_assemble_mpi(f, st4, f, st4, 1, 4, 4, 0, f, nullptr) == MPIV_ERR_ARG);
    EXPECT(mpiv_assemble_mpi_packed(f, st4, f, st4, -1, 4, 4, 2, f, nullptr) == MPIV_ERR_ARG);
    EXPECT(mpiv_assemble_mpi_backward(f, st5, f, st4, f, st4, 1, 4, 4, 2, nullptr, nullptr, nullptr) == MPIV_ERR_ARG);
    EXPECT(mpiv_synth_mpi_packed(1, 4, 4, 3, 3, f, nullptr) == MPIV_ERR_ARG);
    EXPECT(mpiv_probe_gather(f, 16384, 0, 1, f, nullptr) == MPIV_ERR_ARG);
    EXPECT(mpiv_probe_gather(f, 4096, 1, 1, f, nullptr) == MPIV_ERR_ARG);
    EXPECT(mpiv_selftest_div_const(0, nullptr, nullptr) == MPIV_ERR_ARG);
    // debug options
    EXPECT(mpiv_debug_set("render_mv", 1) == MPIV_OK);
    EXPECT(mpiv_debug_set("reset", 0) == MPIV_OK);
    EXPECT(mpiv_debug_set("nope", 1) == MPIV_ERR_ARG);
    EXPECT(mpiv_debug_set(nullptr, 1) == MPIV_ERR_ARG);
    // the host homography chain on exact-size heap buffers (ASan catches any overrun)
    const int B = 3, P = 7;
    std::vector<float> pose(B * 16, 0.f), depths(P), K(B * 9, 0.f), Ki(B * 9, 0.f), H(B * P * 9);
    for (int b = 0; b < B; ++b) {
        for (int i = 0; i < 4; ++i) pose[b * 16 + i * 5] = 1.f;
        pose[b * 16 + 3] = 0.05f * b;
        pose[b * 16 + 11] = -0.02f;
        K[b * 9 + 0] = K[b * 9 + 4] = 100.f + b;
        K[b * 9 + 2] = 32.f;
        K[b * 9 + 5] = 24.f;
        K[b * 9 + 8] = 1.f;
        Ki[b * 9 + 0] = Ki[b * 9 + 4] = 1.f / (100.f + b);
        Ki[b * 9 + 2] = -32.f / (100.f + b);
        Ki[b * 9 + 5] = -24.f / (100.f + b);
        Ki[b * 9 + 8] = 1.f;
    }
    for (int p = 0; p < P; ++p) depths[p] = 100.f / (1 + p);
    EXPECT(mpiv_render_homographies(pose.data(), depths.data(), K.data(), Ki.data(), B, P, H.data()) == MPIV_OK);
    bool finite = true;
    for (float v : H) finite = finite && std::isfinite(v);
    EXPECT(finite);
    EXPECT(mpiv_render_homographies(pose.data(), depths.data(), K.data(), Ki.data(), 0, P, H.data()) == MPIV_ERR_ARG);
    std::printf("abi_check: %d failure(s)\n", failures);
    return failures ? 1 : 0;
}
