// geometry.hip -- per-point projective-geometry helpers of the reference, for callers
// that use them directly (the render / PSV kernels fuse the same arithmetic):
//   transform_points_torch      utils.py:69-88    points @ H^T   (MKL sgemm FMA order)
//   normalize_homogeneous_torch utils.py:90-101   uv / w, w == 0 -> 1e-8 (written back,
//                                                 like the reference's in-place `+=`)
//   pixel2cam_torch             utils.py:356-375  (Ki @ pix) * depth [, 1]
//   cam2pixel_torch             utils.py:377-393  (proj @ cam)[:2] / (z + 1e-10)
#include "mpiv_common.hpp"

namespace mpiv {

// points [M][n][3] contiguous, homs [M][9] -> out [M][n][3]
__global__ __launch_bounds__(256) void transform_points_kernel(const float* __restrict__ pts, int64_t n,
                                                               const float* __restrict__ homs,
                                                               float* __restrict__ out) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int m = blockIdx.y;
    if (i >= n) return;
    const float* h = homs + (int64_t)m * 9;
    const float* p = pts + ((int64_t)m * n + i) * 3;
    float* o = out + ((int64_t)m * n + i) * 3;
    const float x = p[0], y = p[1], z = p[2];
#pragma unroll
    for (int r = 0; r < 3; ++r) o[r] = __builtin_fmaf(h[3 * r + 2], z, __builtin_fmaf(h[3 * r + 1], y, h[3 * r] * x));
}

// pts [n][k+1] contiguous (k = 1..3) -> out [n][k]; w == 0 is replaced in pts
__global__ __launch_bounds__(256) void normalize_homogeneous_kernel(float* __restrict__ pts, int64_t n, int k,
                                                                    float* __restrict__ out) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    float* p = pts + i * (k + 1);
    float w = p[k];
    if (w == 0.0f) {
        w = w + 1e-8f;
        p[k] = w;
    }
    for (int j = 0; j < k; ++j) out[i * k + j] = div_rn(p[j], w);
}

// depth [B][n], pix [B][3][n], ki [B][9] -> cam [B][3 or 4][n]
__global__ __launch_bounds__(256) void pixel2cam_kernel(const float* __restrict__ depth,
                                                        const float* __restrict__ pix, const float* __restrict__ ki,
                                                        int64_t n, int homogeneous, float* __restrict__ cam) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int b = blockIdx.y;
    if (i >= n) return;
    const float* k = ki + (int64_t)b * 9;
    const float* pp = pix + (int64_t)b * 3 * n + i;
    const float x = pp[0], y = pp[n], z = pp[2 * n];
    const float d = depth[(int64_t)b * n + i];
    const int rows = homogeneous ? 4 : 3;
    float* c = cam + (int64_t)b * rows * n + i;
#pragma unroll
    for (int r = 0; r < 3; ++r)
        c[r * n] = __builtin_fmaf(k[3 * r + 2], z, __builtin_fmaf(k[3 * r + 1], y, k[3 * r] * x)) * d;
    if (homogeneous) c[3 * n] = 1.0f;
}

// cam [B][4][n], proj [B][16] -> out [B][n][2]
__global__ __launch_bounds__(256) void cam2pixel_kernel(const float* __restrict__ cam,
                                                        const float* __restrict__ proj, int64_t n,
                                                        float* __restrict__ out) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int b = blockIdx.y;
    if (i >= n) return;
    const float* m = proj + (int64_t)b * 16;
    const float* c = cam + (int64_t)b * 4 * n + i;
    const float X = c[0], Y = c[n], Z = c[2 * n], Wc = c[3 * n];
    float r[3];
#pragma unroll
    for (int j = 0; j < 3; ++j)
        r[j] = __builtin_fmaf(m[4 * j + 3], Wc,
                              __builtin_fmaf(m[4 * j + 2], Z, __builtin_fmaf(m[4 * j + 1], Y, m[4 * j] * X)));
    const float den = r[2] + 1e-10f;
    float* o = out + ((int64_t)b * n + i) * 2;
    o[0] = div_rn(r[0], den);
    o[1] = div_rn(r[1], den);
}

// transform_plane_imgs_torch (utils.py:160-195) for arbitrary target points:
// points [M][Ht*Wt][3], homs [M][9] -> normalised [0,1] sample coords [M][Ht*Wt][2]
// (x / (Ht-1), y / (Wt-1) -- the reference's swap), ready for grid_sample_kernel.
__global__ __launch_bounds__(256) void plane_coords_kernel(const float* __restrict__ pts, int64_t n,
                                                           const float* __restrict__ homs, float hm1, float wm1,
                                                           float* __restrict__ coords) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int m = blockIdx.y;
    if (i >= n) return;
    const float* h = homs + (int64_t)m * 9;
    const float* p = pts + ((int64_t)m * n + i) * 3;
    const float x = p[0], y = p[1], z = p[2];
    const float u = __builtin_fmaf(h[2], z, __builtin_fmaf(h[1], y, h[0] * x));
    const float v = __builtin_fmaf(h[5], z, __builtin_fmaf(h[4], y, h[3] * x));
    float w = __builtin_fmaf(h[8], z, __builtin_fmaf(h[7], y, h[6] * x));
    w = (w == 0.0f) ? w + 1e-8f : w;
    float* o = coords + ((int64_t)m * n + i) * 2;
    o[0] = div_rn(div_rn(u, w), hm1);
    o[1] = div_rn(div_rn(v, w), wm1);
}

// preprocess_image_torch (utils.py:334-342): x*2 - 1 == one fma (2x is exact)
__global__ __launch_bounds__(256) void preprocess_kernel(const float* __restrict__ in, int64_t n,
                                                         float* __restrict__ out) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = __builtin_fmaf(2.0f, in[i], -1.0f);
}

// deprocess_image_torch (utils.py:344-352): ((x + 1) / 2) * 255 then torch's CPU
// float -> uint8 cast, which truncates to int32 (cvttss2si: out of range / NaN give
// INT_MIN) and keeps the low byte.
__global__ __launch_bounds__(256) void deprocess_u8_kernel(const float* __restrict__ in, int64_t n,
                                                           uint8_t* __restrict__ out) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const float v = ((in[i] + 1.0f) * 0.5f) * 255.0f;  // /2 == *0.5 exactly
    const int q = (__builtin_fabsf(v) < 2147483648.0f) ? (int)v : (int)0x80000000;
    out[i] = (uint8_t)(q & 0xFF);
}

// Self-check of div_const (mpiv_common.hpp): every fp32 bit pattern x (a grid-strided
// sweep of all 2^32) against the IEEE quotient x / c.  Counts mismatches among finite,
// non-NaN x whose exact quotient matters for a sample position (|x / c| >= 2^-26).
__global__ __launch_bounds__(256) void div_const_selftest_kernel(float c, float rc,
                                                                 unsigned long long* __restrict__ bad) {
    unsigned long long local = 0;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < (1ull << 32); i += stride) {
        const float x = __builtin_bit_cast(float, (unsigned)i);
        if (!__builtin_isfinite(x)) continue;
        const float exact = x / c;
        if (__builtin_fabsf(exact) < 1.4901161e-08f) continue;  // 2^-26
        const float fast = div_const(x, c, rc);
        local += __builtin_bit_cast(unsigned, fast) != __builtin_bit_cast(unsigned, exact);
    }
    if (local) atomicAdd(bad, local);
}

// ---------------------------------------------------------------------------
// per-(view, plane) render homographies: the inv_homography_torch chain (utils.py:44-67,
// via :278-285 -> :255-262 -> :225-229).  The reference evaluates it with torch-CPU ops
// on materialised [P,B,...] tensors; torch's CPU matmul of these tiny matrices rounds as
// plain products summed in ascending k (no FMA; checked against torch for every shape
// of the chain, batch 1..1280) and the rest is elementwise IEEE arithmetic, so the chain
// is restated exactly.  Shared by the host entry and the device kernel (the library
// builds with -ffp-contract=off on both sides; fp32 division is correctly rounded on
// both).  Kinv = torch.inverse(K) comes from the caller (LAPACK).
// ---------------------------------------------------------------------------

// C = A (M x K) @ B (K x N), row-major, sum in ascending k, no fused multiply-add
template <int M, int K, int N>
__host__ __device__ inline void mm(const float* A, const float* B, float* C) {
    for (int i = 0; i < M; ++i)
        for (int j = 0; j < N; ++j) {
            float s = A[i * K] * B[j];
            for (int k = 1; k < K; ++k) s = s + A[i * K + k] * B[k * N + j];
            C[i * N + j] = s;
        }
}

// pose T [4x4] (row-major), plane depth, K and K^-1 [3x3] -> H [3x3]
__host__ __device__ inline void render_hom_chain(const float* T, float depth, const float* Kb, const float* Ki,
                                                 float* H) {
    const float n_hat[3] = {0.0f, 0.0f, 1.0f};
    float rt[9], t[3];  // rot^T (transpose_torch, exact) and t = pose[:3, 3:]
    for (int i = 0; i < 3; ++i) {
        for (int j = 0; j < 3; ++j) rt[i * 3 + j] = T[j * 4 + i];
        t[i] = T[i * 4 + 3];
    }
    float nr[3], c, rtt[3], num0[9], num[9];
    mm<1, 3, 3>(n_hat, rt, nr);     // n_hat @ rot^T
    mm<1, 3, 1>(nr, t, &c);         // (n_hat @ rot^T) @ t
    mm<3, 3, 1>(rt, t, rtt);        // rot^T @ t
    mm<3, 1, 3>(rtt, n_hat, num0);  // (rot^T @ t) @ n_hat
    mm<3, 3, 3>(num0, rt, num);     // ... @ rot^T
    const float a = -depth;
    float den = a - c;
    den = den + (den == 0.0f ? 1e-8f : 0.0f);  // divide_safe_torch, utils.py:38
    float m[9], km[9];
    for (int e = 0; e < 9; ++e) m[e] = rt[e] + num[e] / den;
    mm<3, 3, 3>(Kb, m, km);  // k_s @ (rot^T + num / den)
    mm<3, 3, 3>(km, Ki, H);  // ... @ inverse(k_t)
}

__global__ __launch_bounds__(256) void render_homographies_kernel(const float* __restrict__ pose,
                                                                  const float* __restrict__ depths,
                                                                  const float* __restrict__ K,
                                                                  const float* __restrict__ Kinv, int B, int P,
                                                                  float* __restrict__ H) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (int64_t)B * P) return;
    const int b = (int)(i / P), p = (int)(i % P);
    render_hom_chain(pose + (int64_t)b * 16, depths[p], K + (int64_t)b * 9, Kinv + (int64_t)b * 9, H + i * 9);
}

// ---------------------------------------------------------------------------
// PSV projection (projective_inverse_warp_torch[2], utils.py:428-438, 747-757):
//   proj = [[K_src, 0], [0, 0, 0, 1]] @ pose  (torch.cat of the padded K, then torch.matmul;
// torch's CPU matmul of 4x4 batches rounds as plain products summed in ascending k, like the
// render chain's: tests/test_host.py checks the host entry against torch bit for bit).
// ---------------------------------------------------------------------------
__host__ __device__ inline void psv_proj(const float* Ks, const float* pose, float* proj) {
    float k4[16];
    for (int i = 0; i < 3; ++i) {
        for (int j = 0; j < 3; ++j) k4[i * 4 + j] = Ks[i * 3 + j];
        k4[i * 4 + 3] = 0.0f;
    }
    k4[12] = 0.0f;
    k4[13] = 0.0f;
    k4[14] = 0.0f;
    k4[15] = 1.0f;
    mm<4, 4, 4>(k4, pose, proj);
}

__global__ __launch_bounds__(64) void psv_proj_kernel(const float* __restrict__ Ks, int64_t ks_bstride,
                                                      const float* __restrict__ pose, int B,
                                                      float* __restrict__ proj) {
    const int b = blockIdx.x * 64 + threadIdx.x;
    if (b < B) psv_proj(Ks + (int64_t)b * ks_bstride, pose + (int64_t)b * 16, proj + (int64_t)b * 16);
}

}  // namespace mpiv
