// sweep.hip -- plane-sweep volume construction and the generic bilinear sampler
// (plane_sweep_torch / _one / _one2 and projective_inverse_warp_torch[2],
// utils.py:409-533, 725-799; bilinear_wrapper_torch / resampler_wrapper_torch,
// utils.py:104-134, 395-407) for gfx950.
//
// PSV: the output [B, Ht, Wt, D*C] is written with consecutive work-items on
// consecutive (depth, channel) words of the same pixel, so each wave stores one
// contiguous run of the volume (the kernel is write-bound: the volume is D times the
// source).  The reference's per-depth Python loop, its per-depth grids and the final
// torch.cat (26% of its time) disappear: one launch writes the whole volume.
#include "mpiv_common.hpp"

namespace mpiv {

struct ImgStrides {
    int64_t b, y, x, c;  // element strides of an NHWC image
};

struct SweepParams {
    int B, Hs, Ws, C, D, Ht, Wt;
    float fhs, fws, half_ws, half_hs;
};

// per-target-pixel camera ray Ki @ (x, y, 1)  (pixel2cam_torch, utils.py:370: MKL
// sgemm FMA order)
__device__ __forceinline__ void ray(const float* __restrict__ k, float fx, float fy, float& rx, float& ry,
                                    float& rz) {
    rx = __builtin_fmaf(k[1], fy, k[0] * fx) + k[2];
    ry = __builtin_fmaf(k[4], fy, k[3] * fx) + k[5];
    rz = __builtin_fmaf(k[7], fy, k[6] * fx) + k[8];
}

// depth d along the ray -> source sample position (utils.py:370 `* depth`,
// cam2pixel_torch :388-391, then (xy + 0.5) / [H, W] SWAPPED :444, grid :406)
__device__ __forceinline__ void sweep_pos(const float* __restrict__ m, float rx, float ry, float rz, float dep,
                                          const SweepParams& sp, float& px, float& py) {
    const float X = rx * dep, Y = ry * dep, Z = rz * dep;
    const float pu = __builtin_fmaf(m[2], Z, __builtin_fmaf(m[1], Y, m[0] * X)) + m[3];
    const float pv = __builtin_fmaf(m[6], Z, __builtin_fmaf(m[5], Y, m[4] * X)) + m[7];
    const float pz = __builtin_fmaf(m[10], Z, __builtin_fmaf(m[9], Y, m[8] * X)) + m[11];
    const float den = pz + 1e-10f;
    const float sx = div_rn(pu, den), sy = div_rn(pv, den);
    const float cx = div_rn(sx + 0.5f, sp.fhs);  // SWAPPED: x / H
    const float cy = div_rn(sy + 0.5f, sp.fws);  //          y / W
    px = unnormalize(to_grid(cx), sp.half_ws);
    py = unnormalize(to_grid(cy), sp.half_hs);
}

__device__ __forceinline__ float ld_img(const float* __restrict__ img, const ImgStrides& s, int ix, int iy, int c,
                                        bool ok) {
    return ok ? img[(int64_t)iy * s.y + (int64_t)ix * s.x + (int64_t)c * s.c] : 0.0f;
}

// one work-item = one (pixel, depth) pair, (d fastest) -> C output words
__global__ __launch_bounds__(256) void plane_sweep_kernel(const float* __restrict__ img, ImgStrides s,
                                                          SweepParams sp, const float* __restrict__ ki,
                                                          const float* __restrict__ proj,
                                                          const float* __restrict__ depths,
                                                          float* __restrict__ out) {
    const int64_t per_view = (int64_t)sp.Ht * sp.Wt * sp.D;
    const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int b = blockIdx.y;
    if (gid >= per_view) return;
    const int d = (int)(gid % sp.D);
    const int64_t pix = gid / sp.D;
    const int y = (int)(pix / sp.Wt), x = (int)(pix % sp.Wt);
    float rx, ry, rz;
    ray(ki + (int64_t)b * 9, (float)x, (float)y, rx, ry, rz);
    float px, py;
    sweep_pos(proj + (int64_t)b * 16, rx, ry, rz, depths[d], sp, px, py);
    const Bilinear bl = bilinear_setup(px, py, sp.Ws, sp.Hs);
    const bool m00 = bl.x0 & bl.y0, m10 = bl.x1 & bl.y0, m01 = bl.x0 & bl.y1, m11 = bl.x1 & bl.y1;
    const float* src = img + (int64_t)b * s.b;
    float* o = out + ((int64_t)b * per_view + gid) * sp.C;
    for (int c = 0; c < sp.C; ++c) {
        o[c] = blend4(bl, ld_img(src, s, bl.ix, bl.iy, c, m00), ld_img(src, s, bl.ix + 1, bl.iy, c, m10),
                      ld_img(src, s, bl.ix, bl.iy + 1, c, m01), ld_img(src, s, bl.ix + 1, bl.iy + 1, c, m11));
    }
}

// Source images padded to 16-B texels: [B][Hs*Ws] float4, channels >= C zero.
__global__ __launch_bounds__(256) void pad_texels_kernel(const float* __restrict__ img, ImgStrides s, int Hs,
                                                         int Ws, int C, float4* __restrict__ out) {
    const int64_t npix = (int64_t)Hs * Ws;
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int b = blockIdx.y;
    if (i >= npix) return;
    const int y = (int)(i / Ws), x = (int)(i % Ws);
    const float* t = img + b * s.b + y * s.y + x * s.x;
    float v[4] = {0.f, 0.f, 0.f, 0.f};
    for (int c = 0; c < C && c < 4; ++c) v[c] = t[c * s.c];
    out[b * npix + i] = make_float4(v[0], v[1], v[2], v[3]);
}

// Plane sweep over padded 16-B texels (C <= 4): four 16-B buffer loads per sample
// with out-of-range taps zeroed by the buffer unit, and the two launch-constant
// divisions (x / Hs, y / Ws) through div_const (FAST, Hs and Ws >= 1 always hold).
// Work-items are (pixel, depth) with depth fastest, so a wave's C-float results are
// one contiguous run of the volume.
constexpr int kSweepILP = 4;       // (pixel, depth) items per work-item, loads issued together
constexpr int kSweepMaxLdsD = 1024; // depths staged in LDS up to this many planes

template <int C>
__global__ __launch_bounds__(256) void plane_sweep_rgba_kernel(const float4* __restrict__ img4, SweepParams sp,
                                                               float rc_hs, float rc_ws, FastDiv fd_d, FastDiv fd_w,
                                                               const float* __restrict__ ki,
                                                               const float* __restrict__ proj,
                                                               const float* __restrict__ depths,
                                                               float* __restrict__ out, int64_t out_bstride,
                                                               int out_pstride) {
    __shared__ float s_dep[kSweepMaxLdsD];
    const bool lds_dep = sp.D <= kSweepMaxLdsD;
    if (lds_dep)
        for (int i = threadIdx.x; i < sp.D; i += blockDim.x) s_dep[i] = depths[i];
    __syncthreads();
    const unsigned per_view = (unsigned)sp.Ht * sp.Wt * sp.D;  // < 2^31, checked on the host
    const int b = blockIdx.y;
    const float* k9 = ki + (int64_t)b * 9;
    const float* m = proj + (int64_t)b * 16;
    const __amdgpu_buffer_rsrc_t r = make_rsrc(img4 + (int64_t)b * sp.Hs * sp.Ws, sp.Hs * sp.Ws * 16);
    // output element of (pixel, d, c): b*out_bstride + pixel*out_pstride + d*C + c
    // (out_pstride = D*C for a bare volume; larger when writing into a wider tensor,
    // e.g. format_network_input_torch's concatenated channels)
    float* ob = out + (int64_t)b * out_bstride;
    const unsigned base = blockIdx.x * (blockDim.x * kSweepILP) + threadIdx.x;
    TapSet t[kSweepILP];
    // phase 1: coordinates + tap loads of all items (kSweepILP x 4 loads in flight)
#pragma unroll
    for (int k = 0; k < kSweepILP; ++k) {
        const unsigned gid = base + k * blockDim.x;
        const bool live = gid < per_view;
        const unsigned g = live ? gid : 0;
        const unsigned pix = fast_div(g, fd_d);
        const int d = (int)(g - pix * sp.D);
        const unsigned yy = fast_div(pix, fd_w);
        const float fy = (float)(int)yy, fx = (float)(int)(pix - yy * sp.Wt);
        float rx, ry, rz;
        ray(k9, fx, fy, rx, ry, rz);
        const float dep = lds_dep ? s_dep[d] : depths[d];
        const float X = rx * dep, Y = ry * dep, Z = rz * dep;
        const float pu = __builtin_fmaf(m[2], Z, __builtin_fmaf(m[1], Y, m[0] * X)) + m[3];
        const float pv = __builtin_fmaf(m[6], Z, __builtin_fmaf(m[5], Y, m[4] * X)) + m[7];
        const float pz = __builtin_fmaf(m[10], Z, __builtin_fmaf(m[9], Y, m[8] * X)) + m[11];
        const float den = pz + 1e-10f;
        const float cx = div_const(div_rn(pu, den) + 0.5f, sp.fhs, rc_hs);  // SWAPPED: x / H, utils.py:444
        const float cy = div_const(div_rn(pv, den) + 0.5f, sp.fws, rc_ws);  //          y / W
        issue_taps(r, sp.Ws, sp.Hs, unnormalize(to_grid(cx), sp.half_ws), unnormalize(to_grid(cy), sp.half_hs),
                   live, t[k]);
    }
    // phase 2: blend + coalesced stores (consecutive work-items = consecutive depths)
#pragma unroll
    for (int k = 0; k < kSweepILP; ++k) {
        const unsigned gid = base + k * blockDim.x;
        const f32x4 v = blend_taps(t[k]);
        if (gid < per_view) {
            const unsigned pix = fast_div(gid, fd_d);
            float* o = ob + (int64_t)pix * out_pstride + (gid - pix * sp.D) * C;
#pragma unroll
            for (int c = 0; c < C; ++c) o[c] = v[c];
        }
    }
}

// projective_inverse_warp_torch[2] with a per-pixel depth map [B, Ht, Wt] (any
// strides) -> [B, Ht, Wt, C]
__global__ __launch_bounds__(256) void inverse_warp_kernel(const float* __restrict__ img, ImgStrides s,
                                                           SweepParams sp, const float* __restrict__ ki,
                                                           const float* __restrict__ proj,
                                                           const float* __restrict__ depth, int64_t dsb,
                                                           int64_t dsy, int64_t dsx, float* __restrict__ out) {
    const int64_t npix = (int64_t)sp.Ht * sp.Wt;
    const int64_t pix = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int b = blockIdx.y;
    if (pix >= npix) return;
    const int y = (int)(pix / sp.Wt), x = (int)(pix % sp.Wt);
    float rx, ry, rz;
    ray(ki + (int64_t)b * 9, (float)x, (float)y, rx, ry, rz);
    float px, py;
    sweep_pos(proj + (int64_t)b * 16, rx, ry, rz, depth[b * dsb + y * dsy + x * dsx], sp, px, py);
    const Bilinear bl = bilinear_setup(px, py, sp.Ws, sp.Hs);
    const bool m00 = bl.x0 & bl.y0, m10 = bl.x1 & bl.y0, m01 = bl.x0 & bl.y1, m11 = bl.x1 & bl.y1;
    const float* src = img + (int64_t)b * s.b;
    float* o = out + ((int64_t)b * npix + pix) * sp.C;
    for (int c = 0; c < sp.C; ++c) {
        o[c] = blend4(bl, ld_img(src, s, bl.ix, bl.iy, c, m00), ld_img(src, s, bl.ix + 1, bl.iy, c, m10),
                      ld_img(src, s, bl.ix, bl.iy + 1, c, m01), ld_img(src, s, bl.ix + 1, bl.iy + 1, c, m11));
    }
}

// ---------------------------------------------------------------------------
// generic sampler: input [N, C, Hi, Wi] (element strides), coords [N, Ho, Wo, 2]
// (element strides) in [0, 1] units, output strides (N, C, H, W) chosen by the
// caller (NCHW for bilinear_wrapper_torch, NHWC for resampler_wrapper_torch).
// ---------------------------------------------------------------------------

struct Strides4 {
    int64_t n, c, y, x;
};

__global__ __launch_bounds__(256) void grid_sample_kernel(const float* __restrict__ in, Strides4 is, int C, int Hi,
                                                          int Wi, const float* __restrict__ coords, Strides4 cs,
                                                          int Ho, int Wo, float* __restrict__ out, Strides4 os) {
    const int64_t npix = (int64_t)Ho * Wo;
    const int64_t pix = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int n = blockIdx.y;
    if (pix >= npix) return;
    const int y = (int)(pix / Wo), x = (int)(pix % Wo);
    const float* cp = coords + n * cs.n + y * cs.y + x * cs.x;
    const float px = unnormalize(to_grid(cp[0]), (float)Wi * 0.5f);
    const float py = unnormalize(to_grid(cp[cs.c]), (float)Hi * 0.5f);
    const Bilinear bl = bilinear_setup(px, py, Wi, Hi);
    const bool m00 = bl.x0 & bl.y0, m10 = bl.x1 & bl.y0, m01 = bl.x0 & bl.y1, m11 = bl.x1 & bl.y1;
    const float* src = in + n * is.n;
    float* o = out + n * os.n + y * os.y + x * os.x;
    const int64_t i00 = (int64_t)bl.iy * is.y + (int64_t)bl.ix * is.x;
    for (int c = 0; c < C; ++c) {
        const float* sc = src + c * is.c;
        const float v00 = m00 ? sc[i00] : 0.f;
        const float v10 = m10 ? sc[i00 + is.x] : 0.f;
        const float v01 = m01 ? sc[i00 + is.y] : 0.f;
        const float v11 = m11 ? sc[i00 + is.y + is.x] : 0.f;
        o[c * os.c] = blend4(bl, v00, v10, v01, v11);
    }
}

// ---------------------------------------------------------------------------
// over_composite (utils.py:136-157) on P layer pointers, each [n, 4] with the same
// element strides (pixel stride ps, channel stride cs) -> [n, 3]
// ---------------------------------------------------------------------------

__global__ __launch_bounds__(256) void over_composite_kernel(const float* const* __restrict__ layers, int P,
                                                             int64_t n, int64_t ps, int64_t chs,
                                                             float* __restrict__ out) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const float* l0 = layers[0] + i * ps;
    float r = l0[0], g = l0[chs], b = l0[2 * chs];
    for (int p = 1; p < P; ++p) {
        const float* l = layers[p] + i * ps;
        const float a = l[3 * chs], om = 1.0f - a;
        r = over(l[0], a, om, r);
        g = over(l[chs], a, om, g);
        b = over(l[2 * chs], a, om, b);
    }
    out[i * 3 + 0] = r;
    out[i * 3 + 1] = g;
    out[i * 3 + 2] = b;
}

}  // namespace mpiv
