// render.hip -- fused projective warp + back-to-front over-composite of an MPI
// (mpi_render_view_torch, utils.py:267-294) for gfx950.
//
// One work-item owns one output pixel of one view and walks the P planes back to
// front, keeping the composited colour in registers: the P warped planes the
// reference materialises (P x [B,H,W,4] plus its grids) never exist.  Homographies
// arrive as a read-only [V][P][9] buffer indexed by wave-uniform (view, plane), so
// they are fetched with scalar loads through the constant cache (no __constant__
// symbol: concurrent streams would race on it).
//
// Two texel layouts:
//  * native  -- the reference's [B,H,W,P,4] tensor, any strides (incl. a stride-0
//               broadcast batch); 4 texel channels are gathered per tap.
//  * packed  -- plane-major [P][H][W] float4 (mpiv_pack_planes).  A wave's 64
//               pixels are one output row, so each of the 4 bilinear taps is one
//               16-B-per-lane load over ~1 KiB of consecutive texels of ONE plane:
//               full 128-B lines, reused by the NE/SE taps and the next row's wave.
#include "mpiv_common.hpp"

namespace mpiv {

constexpr int kTileX = 64;  // one wave = one 64-pixel output row segment
constexpr int kTileY = 4;   // 4 waves per 256-thread block

struct RenderGeom {
    int H, W, P;
    float hm1, wm1, half_w, half_h;
};

__host__ __device__ inline RenderGeom make_geom(int H, int W, int P) {
    RenderGeom g;
    g.H = H; g.W = W; g.P = P;
    g.hm1 = (float)(H - 1);
    g.wm1 = (float)(W - 1);
    g.half_w = (float)W * 0.5f;
    g.half_h = (float)H * 0.5f;
    return g;
}

// ---------------------------------------------------------------------------
// packed plane-major layout
// ---------------------------------------------------------------------------

__device__ __forceinline__ float4 ld_tap(const float4* __restrict__ plane, int W, int ix, int iy, bool ok) {
    float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
    return ok ? plane[(int64_t)iy * W + ix] : z;
}

__device__ __forceinline__ float4 sample_packed(const float4* __restrict__ plane, const RenderGeom& g,
                                                float px, float py) {
    const Bilinear b = bilinear_setup(px, py, g.W, g.H);
    const float4 a = ld_tap(plane, g.W, b.ix, b.iy, b.x0 & b.y0);
    const float4 c = ld_tap(plane, g.W, b.ix + 1, b.iy, b.x1 & b.y0);
    const float4 d = ld_tap(plane, g.W, b.ix, b.iy + 1, b.x0 & b.y1);
    const float4 e = ld_tap(plane, g.W, b.ix + 1, b.iy + 1, b.x1 & b.y1);
    float4 r;
    r.x = blend4(b, a.x, c.x, d.x, e.x);
    r.y = blend4(b, a.y, c.y, d.y, e.y);
    r.z = blend4(b, a.z, c.z, d.z, e.z);
    r.w = blend4(b, a.w, c.w, d.w, e.w);
    return r;
}

// CT = false: final colour [V,H,W,3] (plane p_begin is the back plane; its alpha is
//             ignored, utils.py:152-153).
// CT = true : partial (C, T) for planes [p_begin, p_end) as [V,H,W,4]:
//             C = over-composite of the range onto black, T = prod(1 - a);
//             when `back` is set the range holds plane 0, whose rgb replaces the
//             background (C = rgb0, T = 0).  Ranges combine front-to-back with
//             (Cf, Tf) o (Cb, Tb) = (Cf + Tf*Cb, Tf*Tb)  (SURVEY.md §8e).
template <bool CT>
__global__ __launch_bounds__(256) void render_packed_kernel(const float4* __restrict__ planes,
                                                            int64_t plane_stride, RenderGeom g,
                                                            int p_begin, int p_end, int back,
                                                            const float* __restrict__ homs,
                                                            float* __restrict__ out) {
    const int v = blockIdx.z;
    const int x = blockIdx.x * kTileX + (threadIdx.x & (kWave - 1));
    const int y = blockIdx.y * kTileY + (threadIdx.x >> 6);
    if (x >= g.W || y >= g.H) return;
    const float fx = (float)x, fy = (float)y;
    const float* hv = homs + (int64_t)v * g.P * 9;

    float r = 0.f, gg = 0.f, bb = 0.f, t = 1.f;
    int p = p_begin;
    if (!CT || back) {
        float px, py;
        hom_sample_pos(hv + (int64_t)p * 9, fx, fy, g.hm1, g.wm1, g.half_w, g.half_h, px, py);
        const float4 s = sample_packed(planes + (int64_t)p * plane_stride, g, px, py);
        r = s.x; gg = s.y; bb = s.z; t = 0.f;
        ++p;
    }
    for (; p < p_end; ++p) {
        float px, py;
        hom_sample_pos(hv + (int64_t)p * 9, fx, fy, g.hm1, g.wm1, g.half_w, g.half_h, px, py);
        const float4 s = sample_packed(planes + (int64_t)p * plane_stride, g, px, py);
        const float om = 1.0f - s.w;
        r = over(s.x, s.w, om, r);
        gg = over(s.y, s.w, om, gg);
        bb = over(s.z, s.w, om, bb);
        if (CT) t = t * om;
    }
    const int64_t o = ((int64_t)v * g.H + y) * g.W + x;
    if (CT) {
        reinterpret_cast<float4*>(out)[o] = make_float4(r, gg, bb, t);
    } else {
        out[o * 3 + 0] = r;
        out[o * 3 + 1] = gg;
        out[o * 3 + 2] = bb;
    }
}

// ---------------------------------------------------------------------------
// native [B,H,W,P,C=4] layout, arbitrary element strides
// ---------------------------------------------------------------------------

struct NativeStrides {
    int64_t b, y, x, p, c;
};

__device__ __forceinline__ float ld_nat(const float* __restrict__ base, const NativeStrides& s, int ix, int iy,
                                        int c, bool ok) {
    return ok ? base[(int64_t)iy * s.y + (int64_t)ix * s.x + (int64_t)c * s.c] : 0.0f;
}

__global__ __launch_bounds__(256) void render_native_kernel(const float* __restrict__ mpi, NativeStrides s,
                                                            RenderGeom g, const float* __restrict__ homs,
                                                            float* __restrict__ out) {
    const int v = blockIdx.z;
    const int x = blockIdx.x * kTileX + (threadIdx.x & (kWave - 1));
    const int y = blockIdx.y * kTileY + (threadIdx.x >> 6);
    if (x >= g.W || y >= g.H) return;
    const float fx = (float)x, fy = (float)y;
    const float* hv = homs + (int64_t)v * g.P * 9;
    const float* img = mpi + (int64_t)v * s.b;
    float acc[3] = {0.f, 0.f, 0.f};
    for (int p = 0; p < g.P; ++p) {
        float px, py;
        hom_sample_pos(hv + (int64_t)p * 9, fx, fy, g.hm1, g.wm1, g.half_w, g.half_h, px, py);
        const Bilinear b = bilinear_setup(px, py, g.W, g.H);
        const float* pl = img + (int64_t)p * s.p;
        const bool m00 = b.x0 & b.y0, m10 = b.x1 & b.y0, m01 = b.x0 & b.y1, m11 = b.x1 & b.y1;
        float ch[4];
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            ch[c] = blend4(b, ld_nat(pl, s, b.ix, b.iy, c, m00), ld_nat(pl, s, b.ix + 1, b.iy, c, m10),
                           ld_nat(pl, s, b.ix, b.iy + 1, c, m01), ld_nat(pl, s, b.ix + 1, b.iy + 1, c, m11));
        }
        if (p == 0) {
            acc[0] = ch[0]; acc[1] = ch[1]; acc[2] = ch[2];
        } else {
            const float om = 1.0f - ch[3];
#pragma unroll
            for (int c = 0; c < 3; ++c) acc[c] = over(ch[c], ch[3], om, acc[c]);
        }
    }
    const int64_t o = (((int64_t)v * g.H + y) * g.W + x) * 3;
    out[o + 0] = acc[0];
    out[o + 1] = acc[1];
    out[o + 2] = acc[2];
}

// ---------------------------------------------------------------------------
// layout pack: one view of [H,W,P,C=4] (any strides) -> [P][H][W] float4
// A block moves 64 pixels x 16 planes through LDS so both sides are coalesced:
// reads are 16 planes x 16 B = 256 B per pixel, writes 64 pixels x 16 B = 1 KiB
// per plane.
// ---------------------------------------------------------------------------

constexpr int kPackPix = 64;
constexpr int kPackPl = 16;

__global__ __launch_bounds__(256) void pack_planes_kernel(const float* __restrict__ mpi, NativeStrides s,
                                                          int H, int W, int P, float4* __restrict__ packed,
                                                          int64_t plane_stride) {
    __shared__ float4 tile[kPackPl][kPackPix + 1];
    const int64_t npix = (int64_t)H * W;
    const int64_t pix0 = (int64_t)blockIdx.x * kPackPix;
    const int p0 = blockIdx.y * kPackPl;
    // load: thread -> (pixel i, plane j), plane fastest
    for (int k = threadIdx.x; k < kPackPix * kPackPl; k += blockDim.x) {
        const int j = k % kPackPl, i = k / kPackPl;
        const int64_t pix = pix0 + i;
        const int p = p0 + j;
        float4 val = make_float4(0.f, 0.f, 0.f, 0.f);
        if (pix < npix && p < P) {
            const int yy = (int)(pix / W), xx = (int)(pix % W);
            const float* src = mpi + (int64_t)yy * s.y + (int64_t)xx * s.x + (int64_t)p * s.p;
            if (s.c == 1 && ((reinterpret_cast<uintptr_t>(src) & 15) == 0)) {
                val = *reinterpret_cast<const float4*>(src);
            } else {
                val = make_float4(src[0], src[s.c], src[2 * s.c], src[3 * s.c]);
            }
        }
        tile[j][i] = val;
    }
    __syncthreads();
    // store: thread -> (plane j, pixel i), pixel fastest
    for (int k = threadIdx.x; k < kPackPix * kPackPl; k += blockDim.x) {
        const int i = k % kPackPix, j = k / kPackPix;
        const int64_t pix = pix0 + i;
        const int p = p0 + j;
        if (pix < npix && p < P) packed[(int64_t)p * plane_stride + pix] = tile[j][i];
    }
}

// ---------------------------------------------------------------------------
// ordered combine of plane-range partials (plane sharding)
// parts: G partial [n] float4 (C, T) buffers ordered BACK (index 0) to FRONT.
// out:   [n] x 3 final colour.  Combined front-to-back: acc = part[G-1];
//        acc = (acc.C + acc.T * part[k].C, acc.T * part[k].T) for k = G-2 .. 0.
// ---------------------------------------------------------------------------

__global__ __launch_bounds__(256) void combine_ct_kernel(const float4* __restrict__ parts, int64_t part_stride,
                                                         int G, int64_t n, float* __restrict__ out) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    float4 acc = parts[(int64_t)(G - 1) * part_stride + i];
    for (int k = G - 2; k >= 0; --k) {
        const float4 b = parts[(int64_t)k * part_stride + i];
        acc.x = __builtin_fmaf(acc.w, b.x, acc.x);
        acc.y = __builtin_fmaf(acc.w, b.y, acc.y);
        acc.z = __builtin_fmaf(acc.w, b.z, acc.z);
        acc.w = acc.w * b.w;
    }
    out[i * 3 + 0] = acc.x;
    out[i * 3 + 1] = acc.y;
    out[i * 3 + 2] = acc.z;
}

}  // namespace mpiv
