// render_lds.hip -- the fused warp + over-composite with plane texels staged through
// LDS (A/B variant of the packed-layout render on gfx950, mpiv_render_packed_lds).
//
// Why: the direct kernel (render.hip) gathers four 16-B taps per plane-pixel through
// the vector L1 (64 B per plane-pixel); at ~64 B/clk/CU that data path, not HBM or
// VALU, bounds it (measured 547 G plane-pixel/s = 57-65 B/clk/CU).  Here each block
// stages the source footprint of its output tile once per plane (coalesced 1-KiB
// rows through registers) and the taps become ds_read_b128s.  The footprint of a
// 64x8 tile is ~66x10 texels, so the L1/L2 traffic drops ~2.5x.
//
// Per block (512 threads = 8 waves, one 64-pixel output row per wave):
//  1. prologue: every (plane, tile-corner) pair is pushed through the exact
//     per-pixel recipe; the footprint box of plane p is [floor(min px) - 1,
//     floor(max px) + 2] x (same in y), clipped to [-2, W+1] x [-2, H+1].  Rounded
//     positions are monotone in the exact ones and the exact image of the tile is the
//     convex hull of its corners while w keeps its sign over the tile, so interior
//     pixels land within one texel of the corner box: the margin covers them.
//     Planes whose w changes sign over the tile, whose positions are non-finite, or
//     whose box does not fit the staging buffer are rendered "direct" (global taps).
//  2. loop over planes with two LDS buffers: plane p+1's footprint is loaded into
//     registers while plane p is composited, then written to the other buffer; one
//     barrier per plane.
// Boxes are clipped to the packed planes' 2-texel zero border ([-2, W+1] x [-2, H+1]),
// so every staged texel is real memory and texels outside the image stage as zeros;
// tap indices are clamped into the box, so the LDS path needs no per-tap validity
// test: grid_sample's zero padding falls out.
#include "mpiv_common.hpp"

namespace mpiv {

constexpr int kLTX = 64;           // tile width  (one wave = one output row)
constexpr int kLTY = 8;            // tile height (8 waves)
constexpr int kLThreads = kLTX * kLTY;
constexpr int kLCap = 1024;        // texels per staging buffer (16 KiB)
constexpr int kLMaxP = 510;        // planes per launch in the box table
constexpr int kLMaxPitch = 256;    // footprints wider than this render direct
constexpr int kLDirect = 1;

template <bool CT, bool FAST>
__global__ __launch_bounds__(kLThreads, 8) void render_lds_kernel(const float4* __restrict__ planes,
                                                                  int64_t plane_stride, RenderGeom g, int V,
                                                                  int p_begin, int p_end, int back,
                                                                  const float* __restrict__ homs,
                                                                  float* __restrict__ out) {
    __shared__ __attribute__((aligned(16))) float4 s_tex[2][kLCap];
    __shared__ int4 s_box[kLMaxP];  // per plane: x_lo, y_lo, rows, mode
    __shared__ int s_pitch;

    const int tiles_x = (g.W + kLTX - 1) / kLTX;
    const int lb = xcd_logical_block(blockIdx.x, gridDim.x);
    const int v = lb % V;
    const int tile = lb / V;
    const int tx0 = (tile % tiles_x) * kLTX, ty0 = (tile / tiles_x) * kLTY;
    const int lane = threadIdx.x & (kWave - 1), wave = threadIdx.x >> 6;
    const int x = tx0 + lane, y = ty0 + wave;
    const bool active = x < g.W && y < g.H;
    const float* hv = homs + (int64_t)v * g.P * 9;
    const int np = p_end - p_begin;

    if (threadIdx.x == 0) s_pitch = 0;
    __syncthreads();

    // ---- 1. footprint boxes: thread q -> (plane q/4, corner q%4)
    const int cx1 = min(tx0 + kLTX - 1, g.W - 1), cy1 = min(ty0 + kLTY - 1, g.H - 1);
    for (int q0 = 0; q0 < 4 * np; q0 += kLThreads) {
        const int q = q0 + threadIdx.x;
        const bool live = q < 4 * np;
        const int pl = p_begin + (live ? (q >> 2) : 0);
        const int corner = q & 3;
        const float fx = (float)((corner & 1) ? cx1 : tx0), fy = (float)((corner & 2) ? cy1 : ty0);
        const float* h = hv + (int64_t)pl * 9;
        float px, py;
        render_pos<FAST>(h, fx, fy, g, px, py);
        float w = __builtin_fmaf(h[7], fy, h[6] * fx) + h[8];
        w = (w == 0.0f) ? w + 1e-8f : w;
        const bool fin = __builtin_isfinite(px) && __builtin_isfinite(py) && __builtin_fabsf(px) < 1e7f &&
                         __builtin_fabsf(py) < 1e7f;
        float xmin = floorf(px), xmax = xmin, ymin = floorf(py), ymax = ymin;
        int pos = fin && w > 0.0f, neg = fin && w < 0.0f;
#pragma unroll
        for (int m = 1; m <= 2; m <<= 1) {  // reduce over the 4 corner lanes
            xmin = fminf(xmin, __shfl_xor(xmin, m));
            xmax = fmaxf(xmax, __shfl_xor(xmax, m));
            ymin = fminf(ymin, __shfl_xor(ymin, m));
            ymax = fmaxf(ymax, __shfl_xor(ymax, m));
            pos &= __shfl_xor(pos, m);
            neg &= __shfl_xor(neg, m);
        }
        if (live && corner == 0) {
            int4 bx;
            const bool ok = pos || neg;
            const int xl = ok ? max((int)xmin - 1, -2) : 0, xh = ok ? min((int)xmax + 2, g.W + 1) : 0;
            const int yl = ok ? max((int)ymin - 1, -2) : 0, yh = ok ? min((int)ymax + 2, g.H + 1) : 0;
            const int width = xh - xl + 1, rows = yh - yl + 1;
            bx.x = xl;
            bx.y = yl;
            bx.z = rows;
            bx.w = (!ok || width < 2 || rows < 2 || width > kLMaxPitch || width * rows > kLCap) ? kLDirect : 0;
            s_box[q >> 2] = bx;
            if (bx.w == 0) atomicMax(&s_pitch, width);
        }
    }
    __syncthreads();
    const int pitch = s_pitch;  // common row pitch of the staged footprints

    // this thread's share of a footprint: texels (wave + 8*j)*64 + lane, j = 0, 1, as
    // offsets (in texels) from the box origin in the padded plane
    int rel_j[2];
#pragma unroll
    for (int j = 0; j < 2; ++j) {
        const int idx = (wave + kLTY * j) * kWave + lane;
        const int row = pitch > 0 ? idx / pitch : 0;
        rel_j[j] = row * g.Wp + (idx - row * pitch);
    }

    auto lds_mode = [&](const int4& bx) { return bx.w == 0 && bx.z * pitch <= kLCap; };

    // Register staging: plane p+1's footprint is loaded into registers at the top of
    // iteration p and written to the other LDS buffer after plane p is composited, so
    // its load latency hides behind a whole plane of work.  (LDS-DMA would skip the
    // registers, but hipcc cannot tell which LDS bytes a buffer_load ... lds writes
    // and drains it with vmcnt(0) before every ds_read, serialising the pipeline.)
    // Lanes past the footprint may run off the plane: the buffer range check returns
    // zeros for them and their LDS slots are never read.
    f32x4 stg[2];
    auto fetch = [&](int pl, const int4& bx) {
        const __amdgpu_buffer_rsrc_t r = make_rsrc(planes + (int64_t)pl * plane_stride, g.plane_bytes);
        const int box_org = (bx.y + kPad) * g.Wp + bx.x + kPad;  // >= 0: boxes start at -2
        const int nfp = bx.z * pitch;
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const int base = (wave + kLTY * j) * kWave;  // wave-uniform
            if (base < nfp) stg[j] = llvm_raw_buffer_load_v4f32(r, (box_org + rel_j[j]) * 16, 0, 0);
        }
    };
    auto commit = [&](int buf, const int4& bx) {
        const int nfp = bx.z * pitch;
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const int base = (wave + kLTY * j) * kWave;
            if (base < nfp) *reinterpret_cast<f32x4*>(&s_tex[buf][base + lane]) = stg[j];
        }
    };

    const float fx = (float)x, fy = (float)y;
    float cr = -0.0f, cg = -0.0f, cb = -0.0f, t = 1.0f;
    const bool replace_first = !CT || back;

    int4 bx_next = s_box[0];
    if (lds_mode(bx_next)) {
        fetch(p_begin, bx_next);
        commit(0, bx_next);
    }
    __syncthreads();
    for (int p = p_begin; p < p_end; ++p) {
        const int buf = (p - p_begin) & 1;
        const int4 bx = bx_next;
        const bool more = p + 1 < p_end;
        if (more) {
            bx_next = s_box[p + 1 - p_begin];
            if (lds_mode(bx_next)) fetch(p + 1, bx_next);
        }
        if (active) {
            float px, py;
            render_pos<FAST>(hv + (int64_t)p * 9, fx, fy, g, px, py);
            f32x4 s;
            if (lds_mode(bx)) {
                const float fx0 = floorf(px), fy0 = floorf(py);
                const float wx = px - fx0, ex = 1.0f - wx;
                const float wy = py - fy0, sy = 1.0f - wy;
                TapSet ts;
                ts.nw = sy * ex;
                ts.ne = sy * wx;
                ts.sw = wy * ex;
                ts.se = wy * wx;
                // clamp into the box; past the image (x > W) the clamp stops at W so the
                // taps land in the zero border, never in staged columns that wrapped
                // into the next padded row
                const float ix = __builtin_amdgcn_fmed3f(fx0, (float)bx.x, (float)min(bx.x + pitch - 2, g.W));
                const float iy = __builtin_amdgcn_fmed3f(fy0, (float)bx.y, (float)(bx.y + bx.z - 2));
                // (iy - y_lo) * pitch + (ix - x_lo), exact in fp32 (|values| < 2^24)
                const int li = (int)(__builtin_fmaf(iy, (float)pitch, ix) - (float)(bx.y * pitch + bx.x));
                const float4* st = &s_tex[buf][li];
                ts.a = *reinterpret_cast<const f32x4*>(st);
                ts.b = *reinterpret_cast<const f32x4*>(st + 1);
                ts.c = *reinterpret_cast<const f32x4*>(st + pitch);
                ts.d = *reinterpret_cast<const f32x4*>(st + pitch + 1);
                s = blend_taps(ts);
                // pin the blend inside this branch: if it sinks below the join, the two
                // paths' tap registers merge and hipcc drains vmcnt (the in-flight
                // prefetch) before these ds_reads
                asm volatile("" : "+v"(s));
            } else {
                TapSet ts;
                issue_taps_padded(make_rsrc(planes + (int64_t)p * plane_stride, g.plane_bytes), g.W, g.H, g.Wp,
                                  g.org, g.row, px, py, ts);
                s = blend_taps(ts);
                asm volatile("" : "+v"(s));
            }
            const float a = (replace_first && p == p_begin) ? 1.0f : s[3];
            const float om = 1.0f - a;
            cr = over(s[0], a, om, cr);
            cg = over(s[1], a, om, cg);
            cb = over(s[2], a, om, cb);
            if (CT) t = t * om;
        }
        if (more && lds_mode(bx_next)) commit(buf ^ 1, bx_next);
        __syncthreads();
    }
    if (!active) return;
    const int64_t o = ((int64_t)v * g.H + y) * g.W + x;
    if (CT) {
        reinterpret_cast<float4*>(out)[o] = make_float4(cr, cg, cb, t);
    } else {
        out[o * 3 + 0] = cr;
        out[o * 3 + 1] = cg;
        out[o * 3 + 2] = cb;
    }
}

// The same LDS-staged render reading the reference's own [B,H,W,P,4] tensor in place
// (mpi_render_view_torch without a pack pass; 16-B texels, any element strides with
// contiguous channels).  In that layout a plane's texels are P*16 B apart, so the direct
// kernel gathers one 64-B segment per tap; here each block fetches the footprint of its
// tile once per plane (texels outside the image staged as zeros, the packed layout's
// border made implicit) and the taps are ds_read_b128s.  The 64-B segments a fill
// touches also hold the next 3 planes' texels, which the following fills find in L2 /
// the Infinity Cache.  Planes whose footprint does not fit gather directly.
template <bool FAST>
__global__ __launch_bounds__(kLThreads, 8) void render_lds_native_kernel(const float* __restrict__ mpi,
                                                                         NativeStrides s, RenderGeom g, int V,
                                                                         const float* __restrict__ homs,
                                                                         float* __restrict__ out) {
    __shared__ __attribute__((aligned(16))) float4 s_tex[2][kLCap];
    __shared__ int4 s_box[kLMaxP];  // per plane: x_lo, y_lo, rows, mode
    __shared__ int s_pitch;

    const int tiles_x = (g.W + kLTX - 1) / kLTX;
    const int lb = xcd_logical_block(blockIdx.x, gridDim.x);
    const int v = lb % V;
    const int tile = lb / V;
    const int tx0 = (tile % tiles_x) * kLTX, ty0 = (tile / tiles_x) * kLTY;
    const int lane = threadIdx.x & (kWave - 1), wave = threadIdx.x >> 6;
    const int x = tx0 + lane, y = ty0 + wave;
    const bool active = x < g.W && y < g.H;
    const float* hv = homs + (int64_t)v * g.P * 9;
    const float* img = mpi + (int64_t)v * s.b;
    const int np = g.P;

    if (threadIdx.x == 0) s_pitch = 0;
    __syncthreads();

    // ---- footprint boxes (render_lds_kernel's prologue)
    const int cx1 = min(tx0 + kLTX - 1, g.W - 1), cy1 = min(ty0 + kLTY - 1, g.H - 1);
    for (int q0 = 0; q0 < 4 * np; q0 += kLThreads) {
        const int q = q0 + threadIdx.x;
        const bool live = q < 4 * np;
        const int pl = live ? (q >> 2) : 0;
        const int corner = q & 3;
        const float fx = (float)((corner & 1) ? cx1 : tx0), fy = (float)((corner & 2) ? cy1 : ty0);
        const float* h = hv + (int64_t)pl * 9;
        float px, py;
        render_pos<FAST>(h, fx, fy, g, px, py);
        float w = __builtin_fmaf(h[7], fy, h[6] * fx) + h[8];
        w = (w == 0.0f) ? w + 1e-8f : w;
        const bool fin = __builtin_isfinite(px) && __builtin_isfinite(py) && __builtin_fabsf(px) < 1e7f &&
                         __builtin_fabsf(py) < 1e7f;
        float xmin = floorf(px), xmax = xmin, ymin = floorf(py), ymax = ymin;
        int pos = fin && w > 0.0f, neg = fin && w < 0.0f;
#pragma unroll
        for (int m = 1; m <= 2; m <<= 1) {
            xmin = fminf(xmin, __shfl_xor(xmin, m));
            xmax = fmaxf(xmax, __shfl_xor(xmax, m));
            ymin = fminf(ymin, __shfl_xor(ymin, m));
            ymax = fmaxf(ymax, __shfl_xor(ymax, m));
            pos &= __shfl_xor(pos, m);
            neg &= __shfl_xor(neg, m);
        }
        if (live && corner == 0) {
            int4 bx;
            const bool ok = pos || neg;
            const int xl = ok ? max((int)xmin - 1, -2) : 0, xh = ok ? min((int)xmax + 2, g.W + 1) : 0;
            const int yl = ok ? max((int)ymin - 1, -2) : 0, yh = ok ? min((int)ymax + 2, g.H + 1) : 0;
            const int width = xh - xl + 1, rows = yh - yl + 1;
            bx.x = xl;
            bx.y = yl;
            bx.z = rows;
            bx.w = (!ok || width < 2 || rows < 2 || width > kLMaxPitch || width * rows > kLCap) ? kLDirect : 0;
            s_box[q >> 2] = bx;
            if (bx.w == 0) atomicMax(&s_pitch, width);
        }
    }
    __syncthreads();
    const int pitch = s_pitch;

    int row_j[2], col_j[2];
#pragma unroll
    for (int j = 0; j < 2; ++j) {
        const int idx = (wave + kLTY * j) * kWave + lane;
        row_j[j] = pitch > 0 ? idx / pitch : 0;
        col_j[j] = idx - row_j[j] * pitch;
    }
    auto lds_mode = [&](const int4& bx) { return bx.w == 0 && bx.z * pitch <= kLCap; };

    f32x4 stg[2];
    auto fetch = [&](int pl, const int4& bx) {
        const float* plane = img + (int64_t)pl * s.p;
        const int nfp = bx.z * pitch;
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const int base = (wave + kLTY * j) * kWave;  // wave-uniform
            if (base < nfp) {
                const int tx = bx.x + col_j[j], ty = bx.y + row_j[j];
                const bool in = (unsigned)tx < (unsigned)g.W && (unsigned)ty < (unsigned)g.H;
                const int cx = min(max(tx, 0), g.W - 1), cy = min(max(ty, 0), g.H - 1);
                const f32x4 t = *reinterpret_cast<const f32x4*>(plane + (int64_t)cy * s.y + (int64_t)cx * s.x);
                const f32x4 z = {0.f, 0.f, 0.f, 0.f};
                stg[j] = in ? t : z;
            }
        }
    };
    auto commit = [&](int buf, const int4& bx) {
        const int nfp = bx.z * pitch;
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const int base = (wave + kLTY * j) * kWave;
            if (base < nfp) *reinterpret_cast<f32x4*>(&s_tex[buf][base + lane]) = stg[j];
        }
    };

    const float fx = (float)x, fy = (float)y;
    float cr = -0.0f, cg = -0.0f, cb = -0.0f;  // plane 0 replaces it exactly (render.hip)

    int4 bx_next = s_box[0];
    if (lds_mode(bx_next)) {
        fetch(0, bx_next);
        commit(0, bx_next);
    }
    __syncthreads();
    for (int p = 0; p < np; ++p) {
        const int buf = p & 1;
        const int4 bx = bx_next;
        const bool more = p + 1 < np;
        if (more) {
            bx_next = s_box[p + 1];
            if (lds_mode(bx_next)) fetch(p + 1, bx_next);
        }
        if (active) {
            float px, py;
            render_pos<FAST>(hv + (int64_t)p * 9, fx, fy, g, px, py);
            f32x4 sm;
            if (lds_mode(bx)) {
                const float fx0 = floorf(px), fy0 = floorf(py);
                const float wx = px - fx0, ex = 1.0f - wx;
                const float wy = py - fy0, sy = 1.0f - wy;
                TapSet ts;
                ts.nw = sy * ex;
                ts.ne = sy * wx;
                ts.sw = wy * ex;
                ts.se = wy * wx;
                const float ix = __builtin_amdgcn_fmed3f(fx0, (float)bx.x, (float)min(bx.x + pitch - 2, g.W));
                const float iy = __builtin_amdgcn_fmed3f(fy0, (float)bx.y, (float)(bx.y + bx.z - 2));
                const int li = (int)(__builtin_fmaf(iy, (float)pitch, ix) - (float)(bx.y * pitch + bx.x));
                const float4* st = &s_tex[buf][li];
                ts.a = *reinterpret_cast<const f32x4*>(st);
                ts.b = *reinterpret_cast<const f32x4*>(st + 1);
                ts.c = *reinterpret_cast<const f32x4*>(st + pitch);
                ts.d = *reinterpret_cast<const f32x4*>(st + pitch + 1);
                sm = blend_taps(ts);
                asm volatile("" : "+v"(sm));
            } else {  // the direct native gather (render_native_kernel)
                const Bilinear b = bilinear_setup(px, py, g.W, g.H);
                const float* pl = img + (int64_t)p * s.p;
                TapSet t;
                t.nw = b.nw; t.ne = b.ne; t.sw = b.sw; t.se = b.se;
                t.a = ld_texel<true>(pl, s, g.W, g.H, b.ix, b.iy, b.x0 && b.y0);
                t.b = ld_texel<true>(pl, s, g.W, g.H, b.ix + 1, b.iy, b.x1 && b.y0);
                t.c = ld_texel<true>(pl, s, g.W, g.H, b.ix, b.iy + 1, b.x0 && b.y1);
                t.d = ld_texel<true>(pl, s, g.W, g.H, b.ix + 1, b.iy + 1, b.x1 && b.y1);
                sm = blend_taps(t);
                asm volatile("" : "+v"(sm));
            }
            const float a = p == 0 ? 1.0f : sm[3];
            const float om = 1.0f - a;
            cr = over(sm[0], a, om, cr);
            cg = over(sm[1], a, om, cg);
            cb = over(sm[2], a, om, cb);
        }
        if (more && lds_mode(bx_next)) commit(buf ^ 1, bx_next);
        __syncthreads();
    }
    if (!active) return;
    const int64_t o = (((int64_t)v * g.H + y) * g.W + x) * 3;
    out[o + 0] = cr;
    out[o + 1] = cg;
    out[o + 2] = cb;
}

}  // namespace mpiv
