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
//  * packed  -- plane-major [P][H+4][W+4] float4 with a 2-texel zero border
//               (mpiv_pack_planes).  A wave's 64 pixels are one output row, so each
//               of the 4 bilinear taps is one 16-B-per-lane load over ~1 KiB of
//               consecutive texels of ONE plane: full 128-B lines, reused by the
//               NE/SE taps and the next row's wave.  The border makes grid_sample's
//               zero padding free (issue_taps_padded: no per-tap range test).
#include "mpiv_common.hpp"

namespace mpiv {

constexpr int kTileX = 64;  // one wave = one 64-pixel output row segment
constexpr int kTileY = 4;   // 4 waves per 256-thread block

struct RenderGeom {
    int H, W, P;
    int Wp;                     // padded row pitch W + 4 (texels)
    int org;                    // byte offset of texel (0, 0) in a padded plane
    int row;                    // Wp * 16
    int plane_bytes;            // (H+4)*(W+4)*16 (< 2 GiB, checked on the host)
    float hm1, wm1;             // H-1, W-1: the reference's (swapped) normalisers
    float rc_hm1, rc_wm1;       // RN(1/(H-1)), RN(1/(W-1)) for div_const
    float half_w, half_h;       // grid_sample unnormalise scales W/2, H/2
};

inline RenderGeom make_geom(int H, int W, int P) {
    RenderGeom g;
    g.H = H; g.W = W; g.P = P;
    g.Wp = W + 2 * kPad;
    g.row = g.Wp * 16;
    g.org = (kPad * g.Wp + kPad) * 16;
    g.plane_bytes = (int)((int64_t)(H + 2 * kPad) * g.Wp * 16);
    g.hm1 = (float)(H - 1);
    g.wm1 = (float)(W - 1);
    g.rc_hm1 = 1.0f / g.hm1;
    g.rc_wm1 = 1.0f / g.wm1;
    g.half_w = (float)W * 0.5f;
    g.half_h = (float)H * 0.5f;
    return g;
}

// Target pixel through the plane's homography -> source sample position.
// FAST: the two launch-constant divisions use div_const (valid for H, W >= 2).
template <bool FAST>
__device__ __forceinline__ void render_pos(const float* __restrict__ h, float fx, float fy, const RenderGeom& g,
                                           float& px, float& py) {
    if (FAST) {
        const float u = __builtin_fmaf(h[1], fy, h[0] * fx) + h[2];
        const float v = __builtin_fmaf(h[4], fy, h[3] * fx) + h[5];
        const float w = __builtin_fmaf(h[7], fy, h[6] * fx) + h[8];
        float qu, qv;
        divide_safe2(u, v, w, qu, qv);  // divide_safe_torch, utils.py:35-39
        const float cx = div_const(qu, g.hm1, g.rc_hm1);  // SWAPPED x / (H-1), utils.py:188
        const float cy = div_const(qv, g.wm1, g.rc_wm1);  //         y / (W-1)
        px = unnormalize(to_grid(cx), g.half_w);
        py = unnormalize(to_grid(cy), g.half_h);
    } else {
        hom_sample_pos(h, fx, fy, g.hm1, g.wm1, g.half_w, g.half_h, px, py);
    }
}

// one plane's homography, held in SGPRs (wave-uniform scalar loads)
struct Hom9 {
    float h[9];
};

__device__ __forceinline__ Hom9 load_hom(const float* __restrict__ h) {
    Hom9 r;
#pragma unroll
    for (int k = 0; k < 9; ++k) r.h[k] = h[k];
    return r;
}

// render_pos<true>; GUARD: divide_safe2's per-sample range test; without it the caller
// has proven the fast division for the whole tile (div2_rect_safe).
template <bool GUARD>
__device__ __forceinline__ void render_pos_fast(const float* __restrict__ h, float fx, float fy,
                                                const RenderGeom& g, float& px, float& py) {
    const float u = __builtin_fmaf(h[1], fy, h[0] * fx) + h[2];
    const float v = __builtin_fmaf(h[4], fy, h[3] * fx) + h[5];
    const float w = __builtin_fmaf(h[7], fy, h[6] * fx) + h[8];
    float qu, qv;
    if (GUARD)
        divide_safe2(u, v, w, qu, qv);  // divide_safe_torch, utils.py:35-39
    else
        div2_fast(u, v, w, qu, qv);
    const float cx = div_const(qu, g.hm1, g.rc_hm1);  // SWAPPED x / (H-1), utils.py:188
    const float cy = div_const(qv, g.wm1, g.rc_wm1);  //         y / (W-1)
    px = unnormalize(to_grid(cx), g.half_w);
    py = unnormalize(to_grid(cy), g.half_h);
}

// True when div2_safe(u, v, w) holds for every pixel of [x0, x1] x [y0, y1] (integer
// coordinates).  Each computed coordinate, e.g. u = fma(h1, y, RN(h0*x)) + h2, is a chain
// of correctly rounded operations that are each monotone in x (direction: sign of h0)
// and in y (sign of h1), so over the rectangle it takes its extremes at the corners:
// corners with |u|, |v| <= 2^60 and w of one sign inside [2^-60, 2^60] bound every
// interior value exactly (no rounding margin needed).  NaN corners fail the test.
__device__ __forceinline__ bool div2_rect_safe(const float* __restrict__ h, float x0, float x1, float y0,
                                               float y1) {
    bool ok = true, pos = true, neg = true;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        const float fx = (c & 1) ? x1 : x0, fy = (c & 2) ? y1 : y0;
        const float u = __builtin_fmaf(h[1], fy, h[0] * fx) + h[2];
        const float v = __builtin_fmaf(h[4], fy, h[3] * fx) + h[5];
        const float w = __builtin_fmaf(h[7], fy, h[6] * fx) + h[8];
        ok = ok && div2_safe(u, v, w);
        pos = pos && w > 0.0f;
        neg = neg && w < 0.0f;
    }
    return ok && (pos || neg);
}

// True when every sample of the tile [x0, x1] x [y0, y1] (integer pixel coordinates) reads only
// the packed plane's zero border: floor(px) >= W or <= -2 for every pixel (the clamped taps are
// border columns W, W+1 or -2, -1), or the same in y -- with finite positions, so the bilinear
// weights are finite and the sample is exactly +0.  Valid where div2_rect_safe holds for the
// same rectangle.  The bounds are exact: u, v, w are monotone chains whose values over the
// rectangle lie between their corner extremes (div2_rect_safe); with w of one sign, RN(u / w)
// takes its extremes among the four (u, w) extreme pairs (the kernels' fast division equals it
// wherever the quotient can move a position, mpiv_common.hpp div2_rn); div_const, to_grid and
// unnormalize are monotone.  One texel of margin on top.
// Round 6: the reference's swapped normalisation (utils.py:186-188) maps output column x to
// texel column ~x*W/(H-1), so on a landscape MPI every column past ~H samples the border alone:
// 44 % of a config-2 frame (1024 x 576), 47 % of config 5's (4096 x 2160).
__device__ __forceinline__ bool sample_bounds(const float* __restrict__ h, float x0, float x1, float y0, float y1,
                                              const RenderGeom& g, float& px0, float& px1, float& py0, float& py1) {
    float u0 = __builtin_inff(), u1 = -__builtin_inff(), v0 = u0, v1 = u1, w0 = u0, w1 = u1;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        const float fx = (c & 1) ? x1 : x0, fy = (c & 2) ? y1 : y0;
        const float u = __builtin_fmaf(h[1], fy, h[0] * fx) + h[2];
        const float v = __builtin_fmaf(h[4], fy, h[3] * fx) + h[5];
        const float w = __builtin_fmaf(h[7], fy, h[6] * fx) + h[8];
        u0 = fminf(u0, u); u1 = fmaxf(u1, u);
        v0 = fminf(v0, v); v1 = fmaxf(v1, v);
        w0 = fminf(w0, w); w1 = fmaxf(w1, w);
    }
    float qu0 = __builtin_inff(), qu1 = -__builtin_inff(), qv0 = qu0, qv1 = qu1;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        const float w = (c & 2) ? w1 : w0;
        const float qu = div_rn((c & 1) ? u1 : u0, w), qv = div_rn((c & 1) ? v1 : v0, w);
        qu0 = fminf(qu0, qu); qu1 = fmaxf(qu1, qu);
        qv0 = fminf(qv0, qv); qv1 = fmaxf(qv1, qv);
    }
    px0 = unnormalize(to_grid(div_const(qu0, g.hm1, g.rc_hm1)), g.half_w);
    px1 = unnormalize(to_grid(div_const(qu1, g.hm1, g.rc_hm1)), g.half_w);
    py0 = unnormalize(to_grid(div_const(qv0, g.wm1, g.rc_wm1)), g.half_h);
    py1 = unnormalize(to_grid(div_const(qv1, g.wm1, g.rc_wm1)), g.half_h);
    const float big = 0x1p100f;  // finite (|x| < inf, NaN fails) with room to spare
    return __builtin_fabsf(px0) < big && __builtin_fabsf(px1) < big && __builtin_fabsf(py0) < big &&
           __builtin_fabsf(py1) < big;
}

__device__ __forceinline__ bool tile_dead(const float* __restrict__ h, float x0, float x1, float y0, float y1,
                                          const RenderGeom& g) {
    float px0, px1, py0, py1;
    const bool finite = sample_bounds(h, x0, x1, y0, y1, g, px0, px1, py0, py1);
    return finite && (px0 >= (float)(g.W + 1) || px1 < -2.0f || py0 >= (float)(g.H + 1) || py1 < -2.0f);
}

// The texel rows [r0, r1] (r0 > r1: none) that the in-image taps of every output pixel of
// [x0, x1] x [y0, y1] can read for this plane: floor(py) and floor(py) + 1 over sample_bounds'
// exact range, one row of margin each side; the whole image where the division is not provable
// or a bound is not finite.  (mpiv_assemble_mpi_sampled: the rows the fused backward's chain reads.)
__device__ __forceinline__ int2 sampled_rows(const float* __restrict__ h, float x0, float x1, float y0, float y1,
                                             const RenderGeom& g) {
    float px0, px1, py0, py1;
    if (!div2_rect_safe(h, x0, x1, y0, y1) || !sample_bounds(h, x0, x1, y0, y1, g, px0, px1, py0, py1))
        return make_int2(0, g.H - 1);
    if (px0 >= (float)(g.W + 1) || px1 < -2.0f || py0 >= (float)(g.H + 1) || py1 < -2.0f) return make_int2(0, -1);
    const int r0 = (int)floorf(fmaxf(py0, -4.0f)) - 1, r1 = (int)floorf(fminf(py1, (float)(g.H + 4))) + 2;
    return make_int2(max(r0, 0), min(r1, g.H - 1));
}

// A dead tile's pixel (tile_dead): the per-plane over-composite of zero samples, the sampling
// kernels' own update with s = (+0, +0, +0, +0) -- no positions, no gathers.
template <bool CT>
__device__ __forceinline__ void composite_zero(int p_begin, int p_end, bool replace_first, float& cr, float& cg,
                                               float& cb, float& t) {
    for (int p = p_begin; p < p_end; ++p) {
        const float a = (replace_first && p == p_begin) ? 1.0f : 0.0f;
        const float om = 1.0f - a;
        cr = over(0.0f, a, om, cr);
        cg = over(0.0f, a, om, cg);
        cb = over(0.0f, a, om, cb);
        if (CT) t = t * om;
    }
}

// ---------------------------------------------------------------------------
// packed plane-major layout
// ---------------------------------------------------------------------------

// Bijective XCD-aware block order: the dispatcher deals blocks round-robin over the
// 8 XCDs (MI355X_MICROARCH.md §Workgroup dispatch), so hardware block b is given the
// logical id  start(b % 8) + b / 8, i.e. each XCD walks one contiguous range of
// logical ids.  Logical ids enumerate (tile, view) with the VIEW fastest, so the
// views of one output tile -- whose source footprints overlap almost entirely along a
// camera path -- run together on one XCD and share its L2.  Placement only affects
// speed, never correctness.
__device__ __forceinline__ int xcd_logical_block(int b, int nblocks) {
    const int q = nblocks >> 3, r = nblocks & 7;
    const int xcd = b & 7, k = b >> 3;
    return xcd * q + (xcd < r ? xcd : r) + k;
}

// CT = false: final colour [V,H,W,3]; plane p_begin is the back plane, whose alpha is
//             ignored (utils.py:152-153).
// CT = true : partial (C, T) for planes [p_begin, p_end) as [V,H,W,4]:
//             C = over-composite of the range onto black, T = prod(1 - a);
//             with `back` set the range holds plane 0, whose rgb replaces the
//             background (C = rgb0, T = 0).  Ranges combine front-to-back with
//             (Cf, Tf) o (Cb, Tb) = (Cf + Tf*Cb, Tf*Tb)  (SURVEY.md §8e).
// One work-item = one output pixel of one view.  Plane p+1's four tap loads are
// issued before plane p is blended, so every wave keeps 8 x 16 B in flight.
// MODE 0: generic recipe (H or W < 2); 1: fast recipe with the per-sample division
// guard; 2: fast recipe, fast division proven for the block's tile and every plane.
template <bool CT, int MODE>
__device__ __forceinline__ void render_packed_pixel(const float4* __restrict__ planes, int64_t plane_stride,
                                                    const RenderGeom& g, int p_begin, int p_end, int back,
                                                    const float* __restrict__ hv, int x, int y,
                                                    float* __restrict__ out_px) {
    const float fx = (float)x, fy = (float)y;
    // The reference's plane 0 replaces the background: with alpha forced to 1 and the
    // colour started at -0.0, `out = rgb*1 + (-0)*(1-1)` returns rgb bit for bit (x + -0
    // == x for every x, signed zeros included), so every plane runs the same code.
    float cr = -0.0f, cg = -0.0f, cb = -0.0f, t = 1.0f;
    const bool replace_first = !CT || back;
    const int last = p_end - 1;
    // plane p's taps; past the range the last plane is re-issued (L2-hot, result
    // unused) so every iteration issues unconditionally and the compiler can count
    // vmcnt exactly
    // the homography of plane p is fetched (scalar loads) a full iteration ahead, so its
    // latency hides behind two blends instead of stalling the issue that uses it
    auto hom = [&](int p) { return load_hom(hv + (int64_t)(p < last ? p : last) * 9); };
    auto issue = [&](int p, const Hom9& h, TapSet& ts) {
        const int q = p < last ? p : last;
        float px, py;
        if (MODE == 0)
            render_pos<false>(h.h, fx, fy, g, px, py);
        else
            render_pos_fast<MODE == 1>(h.h, fx, fy, g, px, py);
        issue_taps_padded(make_rsrc(planes + (int64_t)q * plane_stride, g.plane_bytes), g.W, g.H, g.Wp, g.org,
                          g.row, px, py, ts);
    };
    auto consume = [&](const TapSet& ts, bool first) {
        const f32x4 s = blend_taps(ts);
        const float a = first ? 1.0f : s[3];
        const float om = 1.0f - a;
        cr = over(s[0], a, om, cr);
        cg = over(s[1], a, om, cg);
        cb = over(s[2], a, om, cb);
        if (CT) t = t * om;
    };
    // ping-pong between two tap sets (no register rotation): the next plane's loads
    // are in flight while the current one is blended.  sched_barrier keeps each issue
    // block ahead of the previous plane's blend.
    // Loop invariant: at the top of every iteration exactly A's four loads are in
    // flight (no mid-loop exits), so the compiler's vmcnt bookkeeping stays exact.
    TapSet A, B;
    Hom9 hA = hom(p_begin), hB = hom(p_begin + 1);
    issue(p_begin, hA, A);
    hA = hom(p_begin + 2);
    int p = p_begin;
    for (; p + 1 < p_end; p += 2) {  // A holds plane p, B will hold p + 1
        issue(p + 1, hB, B);
        hB = hom(p + 3);  // used one iteration later
        __builtin_amdgcn_sched_barrier(0);
        consume(A, replace_first && p == p_begin);
        issue(p + 2, hA, A);
        hA = hom(p + 4);
        __builtin_amdgcn_sched_barrier(0);
        consume(B, false);
    }
    if (p < p_end) consume(A, replace_first && p == p_begin);
    if (CT) {
        *reinterpret_cast<float4*>(out_px) = make_float4(cr, cg, cb, t);
    } else {
        out_px[0] = cr;
        out_px[1] = cg;
        out_px[2] = cb;
    }
}

template <bool CT, bool FAST>
__global__ __launch_bounds__(256) void render_packed_kernel(const float4* __restrict__ planes,
                                                            int64_t plane_stride, RenderGeom g, int V,
                                                            int p_begin, int p_end, int back,
                                                            const float* __restrict__ homs,
                                                            float* __restrict__ out) {
    const int tiles_x = (g.W + kTileX - 1) / kTileX;
    const int lb = xcd_logical_block(blockIdx.x, gridDim.x);
    const int v = lb % V;
    const int tile = lb / V;
    const int tx0 = (tile % tiles_x) * kTileX, ty0 = (tile / tiles_x) * kTileY;
    const int x = tx0 + (threadIdx.x & (kWave - 1));
    const int y = ty0 + (threadIdx.x >> 6);
    const float* hv = homs + (int64_t)v * g.P * 9;
    // block prologue: prove the fast division for the tile, all planes at once
    bool proven = false, dead = false;
    if (FAST) {
        const float x0 = (float)tx0, x1 = (float)min(tx0 + kTileX - 1, g.W - 1);
        const float y0 = (float)ty0, y1 = (float)min(ty0 + kTileY - 1, g.H - 1);
        bool ok = true, dd = true;
        for (int p = p_begin + (int)threadIdx.x; p < p_end; p += 256) {
            const float* hp = hv + (int64_t)p * 9;
            const bool safe = div2_rect_safe(hp, x0, x1, y0, y1);
            ok = ok && safe;
            dd = dd && safe && tile_dead(hp, x0, x1, y0, y1, g);
        }
        proven = __syncthreads_and(ok);
        dead = __syncthreads_and(dd);
    }
    if (x >= g.W || y >= g.H) return;
    const int64_t o = ((int64_t)v * g.H + y) * g.W + x;
    float* out_px = CT ? out + o * 4 : out + o * 3;
    if (dead) {  // every plane samples the zero border over the whole tile
        float cr = -0.0f, cg = -0.0f, cb = -0.0f, t = 1.0f;
        composite_zero<CT>(p_begin, p_end, !CT || back, cr, cg, cb, t);
        if (CT) {
            *reinterpret_cast<float4*>(out_px) = make_float4(cr, cg, cb, t);
        } else {
            out_px[0] = cr;
            out_px[1] = cg;
            out_px[2] = cb;
        }
        return;
    }
    if (!FAST)
        render_packed_pixel<CT, 0>(planes, plane_stride, g, p_begin, p_end, back, hv, x, y, out_px);
    else if (proven)
        render_packed_pixel<CT, 2>(planes, plane_stride, g, p_begin, p_end, back, hv, x, y, out_px);
    else
        render_packed_pixel<CT, 1>(planes, plane_stride, g, p_begin, p_end, back, hv, x, y, out_px);
}

// ---------------------------------------------------------------------------
// R vertically adjacent pixels per work-item, planes outermost (render_rows_kernel)
// ---------------------------------------------------------------------------
//
// With one view per launch every texel crosses HBM about once, plus the halo its
// neighbouring tiles re-read: a 64x4 tile's footprint is ~66x6 texels per plane, and
// those re-reads come back from HBM/MALL whenever the neighbour reaches the plane
// later than the L2 can hold it.  Here a lane renders rows y .. y+R-1 of its column
// and the plane loop is outside the row loop, so row k+1's north taps are row k's
// south taps fetched moments earlier by the same wave (an L1/L2 hit): a block tile of
// 64 x 4R re-reads only its outer halo.  Same per-sample recipe as
// render_packed_pixel, two samples in flight (ping-pong across rows and planes).
template <bool CT, bool GUARD, int R>
__device__ __forceinline__ void render_rows_pixels(const float4* __restrict__ planes, int64_t plane_stride,
                                                   const RenderGeom& g, int p_begin, int p_end, int back,
                                                   const float* __restrict__ hv, int x, int y0,
                                                   float* cr, float* cg, float* cb, float* tt) {
    static_assert(R % 2 == 0, "R must be even");
    const float fx = (float)x;
    const bool replace_first = !CT || back;
    const int last = p_end - 1;
    auto hom = [&](int p) { return load_hom(hv + (int64_t)(p < last ? p : last) * 9); };
    auto issue = [&](int p, int k, const Hom9& h, TapSet& ts) {
        const int q = p < last ? p : last;
        float px, py;
        render_pos_fast<GUARD>(h.h, fx, (float)(y0 + k), g, px, py);
        issue_taps_padded(make_rsrc(planes + (int64_t)q * plane_stride, g.plane_bytes), g.W, g.H, g.Wp, g.org,
                          g.row, px, py, ts);
    };
    auto consume = [&](const TapSet& ts, int k, bool first) {
        const f32x4 s = blend_taps(ts);
        const float a = first ? 1.0f : s[3];
        const float om = 1.0f - a;
        cr[k] = over(s[0], a, om, cr[k]);
        cg[k] = over(s[1], a, om, cg[k]);
        cb[k] = over(s[2], a, om, cb[k]);
        if (CT) tt[k] = tt[k] * om;
    };
    TapSet A, B;
    Hom9 h = hom(p_begin), hn = hom(p_begin + 1);
    issue(p_begin, 0, h, A);
    for (int p = p_begin; p < p_end; ++p) {
        const bool first = replace_first && p == p_begin;
#pragma unroll
        for (int k = 0; k < R; k += 2) {  // A holds (p, k)
            issue(p, k + 1, h, B);
            __builtin_amdgcn_sched_barrier(0);
            consume(A, k, first);
            if (k + 2 < R)
                issue(p, k + 2, h, A);
            else
                issue(p + 1, 0, hn, A);  // past the end: the last plane again (cached, unused)
            __builtin_amdgcn_sched_barrier(0);
            consume(B, k + 1, first);
        }
        h = hn;
        hn = hom(p + 2);
    }
}

// The same with VERTICAL TAP SHARING (VS).  Along a lane's R rows the sample usually moves
// down exactly one texel row in the same column (near-identity homographies): then row k's
// north taps ARE row k-1's south taps, the same memory words (the clamped tap offsets are
// compared), already in registers.  Row k always gathers its two south taps and gathers the
// north pair only when some lane of the wave does not continue (a wave-uniform branch; lanes
// that continue get the buffer's zero range there and take the previous row's south taps).
// The texture path charges per wave instruction, so its work drops from 4 to ~2.5 gathers per
// sample on a camera path; the result is bit-identical.
// SAME (round 6, stretched MPIs): the reference's swapped normalisation advances the sample by
// H/(W-1) texel rows per output row -- 0.53 for config 5, 0.56 for config 2 -- so about every other
// row's tap origin does not move at all: then all four of its taps ARE the previous row's (the same
// memory words).  Per row and wave the south pair is gathered as before and the north pair only when
// some lane neither stayed nor moved one row down (a lane that stayed keeps the previous row's north
// taps): 2 gathers per row instead of 4 on most rows of a stretched frame.
template <bool CT, bool GUARD, int R, int D = 2, bool SAME = false, bool OOB = false>
__device__ __forceinline__ void render_rows_vs_pixels(const float4* __restrict__ planes, int64_t plane_stride,
                                                      const RenderGeom& g, int p_begin, int p_end, int back,
                                                      const float* __restrict__ hv, int x, int y0,
                                                      float* cr, float* cg, float* cb, float* tt,
                                                      unsigned& nvm) {
    static_assert(D != 2 || R % 2 == 0, "R must be even");
    static_assert(!SAME || D > 2, "same-row reuse is built on the ring of rows in flight");
    struct RowTaps {
        f32x4 a, b, c, d;  // NW, NE (own, when not shared), SW, SE
        float nw, ne, sw, se;
        int off;           // byte offset of the NW tap in the padded plane
        bool sh;           // NW, NE = the previous row's SW, SE
        bool own;          // wave-uniform: some lane gathered its own north taps
        bool same;         // SAME: all four taps = the previous row's (the origin did not move)
        bool any_same;     // SAME, wave-uniform: some lane's origin did not move
        bool all_same;     // SAME + OOB, wave-uniform: every lane's origin stayed
    };
    const float fx = (float)x;
    const bool replace_first = !CT || back;
    const int last = p_end - 1;
    auto hom = [&](int p) { return load_hom(hv + (int64_t)(p < last ? p : last) * 9); };
    auto issue = [&](int p, int k, const Hom9& h, int prev_off, bool can_share, RowTaps& t) {
        const int q = p < last ? p : last;
        float px, py;
        render_pos_fast<GUARD>(h.h, fx, (float)(y0 + k), g, px, py);
        // issue_taps_padded's weights and clamped offset
        const float fx0 = floorf(px), fy0 = floorf(py);
        const float wx = px - fx0, ex = 1.0f - wx;
        const float wy = py - fy0, sy = 1.0f - wy;
        t.nw = sy * ex;
        t.ne = sy * wx;
        t.sw = wy * ex;
        t.se = wy * wx;
        const int cx = (int)__builtin_amdgcn_fmed3f(fx0, -2.0f, (float)g.W);
        const int cy = (int)__builtin_amdgcn_fmed3f(fy0, -2.0f, (float)g.H);
        const int off = (__mul24(cy, g.Wp) + cx) * 16 + g.org;
        t.off = off;
        t.sh = can_share && off == prev_off + g.row;
        const __amdgpu_buffer_rsrc_t r = make_rsrc(planes + (int64_t)q * plane_stride, g.plane_bytes);
        if constexpr (SAME) {
            // the south pair stays unconditional: a wave that could skip every load of a row makes
            // the compiler's load counting drain the whole ring before each consume (measured 30%
            // slower); a lane whose origin stayed re-reads the previous row's south words (cached).
            // OOB: where every lane stayed, the pair goes to the buffer's out-of-range offset (no
            // memory access, the same instruction count) and the row takes the previous row's taps
            // whole -- one- and two-view launches (config 5's shard 0.57 -> 0.53 ms; with many views
            // the extra live state costs the fourth wave per SIMD, profiles/r06_same_oob_ab/)
            t.same = can_share && off == prev_off;
            t.any_same = __builtin_amdgcn_ballot_w64(t.same) != 0;
            t.all_same = OOB && __builtin_amdgcn_ballot_w64(!t.same) == 0;
            const int soff = t.all_same ? kOOB - 16 : off;
            t.c = llvm_raw_buffer_load_v4f32(r, soff, g.row, 0);
            t.d = llvm_raw_buffer_load_v4f32(r, soff + 16, g.row, 0);
            const bool need_n = !(t.sh || t.same);
            t.own = __builtin_amdgcn_ballot_w64(need_n) != 0;
            nvm += t.own ? 4u : 2u;
            if (t.own) {
                t.a = llvm_raw_buffer_load_v4f32(r, need_n ? off : kOOB, 0, 0);
                t.b = llvm_raw_buffer_load_v4f32(r, (need_n ? off : kOOB - 16) + 16, 0, 0);
            }
            return;
        }
        t.c = llvm_raw_buffer_load_v4f32(r, off, g.row, 0);
        t.d = llvm_raw_buffer_load_v4f32(r, off + 16, g.row, 0);
#ifndef MPIV_VS_ZINIT
#define MPIV_VS_ZINIT 0
#endif
        if (MPIV_VS_ZINIT) {  // defined on both paths (lets the allocator keep one register set)
            t.a = f32x4{0.f, 0.f, 0.f, 0.f};
            t.b = t.a;
        }
        t.own = __builtin_amdgcn_ballot_w64(!t.sh) != 0;
        nvm += t.own ? 4u : 2u;  // gather instructions this wave issues (census builds only)
        if (t.own) {  // wave-uniform: some lane needs its own north taps
            t.a = llvm_raw_buffer_load_v4f32(r, t.sh ? kOOB : off, 0, 0);
            t.b = llvm_raw_buffer_load_v4f32(r, (t.sh ? kOOB - 16 : off) + 16, 0, 0);
        }
    };
    // SAME: the previous row's effective taps (pa, pb, pc, pd) in, this row's out
    auto consume_same = [&](const RowTaps& t, f32x4& pa, f32x4& pb, f32x4& pc, f32x4& pd, int k, bool first) {
        f32x4 na = pc, nb = pd;  // every lane moved one row down: vertical reuse
        f32x4 sc_ = t.c, sd_ = t.d;
        if (OOB && t.all_same) {  // every lane stayed: the previous row's four taps
            na = pa; nb = pb; sc_ = pc; sd_ = pd;
        } else if (t.own || t.any_same) {
            asm volatile("");  // keep the per-lane selects behind this wave-uniform branch
#pragma unroll
            for (int c = 0; c < 4; ++c) {
                na[c] = t.same ? pa[c] : (t.sh ? pc[c] : t.a[c]);
                nb[c] = t.same ? pb[c] : (t.sh ? pd[c] : t.b[c]);
            }
        }
        f32x4 s;
#pragma unroll
        for (int c = 0; c < 4; ++c) {  // blend_taps' fma chain
            float acc = na[c] * t.nw;
            acc = __builtin_fmaf(nb[c], t.ne, acc);
            acc = __builtin_fmaf(sc_[c], t.sw, acc);
            acc = __builtin_fmaf(sd_[c], t.se, acc);
            s[c] = acc;
        }
        const float a = first ? 1.0f : s[3];
        const float om = 1.0f - a;
        cr[k] = over(s[0], a, om, cr[k]);
        cg[k] = over(s[1], a, om, cg[k]);
        cb[k] = over(s[2], a, om, cb[k]);
        if (CT) tt[k] = tt[k] * om;
        asm volatile("" : "+v"(cr[k]), "+v"(cg[k]), "+v"(cb[k]));
        if (CT) asm volatile("" : "+v"(tt[k]));
        pa = na; pb = nb; pc = sc_; pd = sd_;
    };
    auto consume = [&](const RowTaps& t, const f32x4& pc, const f32x4& pd, int k, bool first) {
        f32x4 s;
        f32x4 na = pc, nb = pd;  // every lane continues (the common case): no per-lane select
#ifndef MPIV_VS_BRANCH
#define MPIV_VS_BRANCH 1
#endif
        if (!MPIV_VS_BRANCH || t.own) {
#ifndef MPIV_VS_ASMBR
#define MPIV_VS_ASMBR 1
#endif
            if (MPIV_VS_ASMBR) asm volatile("");  // keeps this a real (wave-uniform) branch: if-converted, its 8 selects ran always
#pragma unroll
            for (int c = 0; c < 4; ++c) {
                na[c] = t.sh ? pc[c] : t.a[c];
                nb[c] = t.sh ? pd[c] : t.b[c];
            }
        }
#pragma unroll
        for (int c = 0; c < 4; ++c) {  // blend_taps' fma chain
            float acc = na[c] * t.nw;
            acc = __builtin_fmaf(nb[c], t.ne, acc);
            acc = __builtin_fmaf(t.c[c], t.sw, acc);
            acc = __builtin_fmaf(t.d[c], t.se, acc);
            s[c] = acc;
        }
        const float a = first ? 1.0f : s[3];
        const float om = 1.0f - a;
        cr[k] = over(s[0], a, om, cr[k]);
        cg[k] = over(s[1], a, om, cg[k]);
        cb[k] = over(s[2], a, om, cb[k]);
        if (CT) tt[k] = tt[k] * om;
        // pin the blend here: IR passes otherwise sink it past the following rows' north-load
        // branches, and every row's taps stay live at once (222 VGPRs)
        asm volatile("" : "+v"(cr[k]), "+v"(cg[k]), "+v"(cb[k]));
        if (CT) asm volatile("" : "+v"(tt[k]));
    };
    f32x4 sc = {0.f, 0.f, 0.f, 0.f}, sd = sc;  // the previous row's south taps
    [[maybe_unused]] f32x4 sa = sc, sb = sc;   // SAME: ... and north taps
    Hom9 h = hom(p_begin), hn = hom(p_begin + 1);
    if constexpr (D != 2) {  // D rows in flight (a ring of D tap sets; A/B)
        static_assert(R % D == 0 && D > 2, "ring depth must divide R");
        RowTaps T[D];
        issue(p_begin, 0, h, 0, false, T[0]);
#pragma unroll
        for (int k = 1; k < D - 1; ++k) issue(p_begin, k, h, T[k - 1].off, true, T[k]);
        for (int p = p_begin; p < p_end; ++p) {
            const bool first = replace_first && p == p_begin;
#pragma unroll
            for (int k = 0; k < R; ++k) {
                const int kk = k + D - 1;  // the row issued now, D - 1 ahead of the one consumed
                if (kk < R)
                    issue(p, kk, h, T[(kk - 1) % D].off, true, T[kk % D]);
                else if (kk == R)
                    issue(p + 1, 0, hn, 0, false, T[kk % D]);  // past the end: the last plane again (unused)
                else
                    issue(p + 1, kk - R, hn, T[(kk - 1) % D].off, true, T[kk % D]);
                asm volatile("" ::: "memory");
                __builtin_amdgcn_sched_barrier(0);
                if constexpr (SAME) {
                    consume_same(T[k % D], sa, sb, sc, sd, k, first);
                } else {
                    consume(T[k % D], sc, sd, k, first);
                    sc = T[k % D].c;
                    sd = T[k % D].d;
                }
            }
            h = hn;
            hn = hom(p + 2);
        }
        return;
    }
    RowTaps A, B;
    issue(p_begin, 0, h, 0, false, A);
    for (int p = p_begin; p < p_end; ++p) {
        const bool first = replace_first && p == p_begin;
#pragma unroll
        for (int k = 0; k < R; k += 2) {  // A holds (p, k)
            issue(p, k + 1, h, A.off, true, B);
            asm volatile("" ::: "memory");  // no later row's loads above this point (IR passes hoist them
            __builtin_amdgcn_sched_barrier(0);  // across the north-load branch otherwise: 222 VGPRs)
            consume(A, sc, sd, k, first);
            sc = A.c;
            sd = A.d;
            if (k + 2 < R)
                issue(p, k + 2, h, B.off, true, A);
            else
                issue(p + 1, 0, hn, 0, false, A);  // past the end: the last plane again (cached, unused)
            asm volatile("" ::: "memory");
            __builtin_amdgcn_sched_barrier(0);
            consume(B, sc, sd, k + 1, first);
            sc = B.c;
            sd = B.d;
        }
        h = hn;
        hn = hom(p + 2);
    }
}

// The same with the R rows' compositing state kept in LDS (rows loop not unrolled: the
// register footprint of one sample in flight, so occupancy stays high for large R).
// state: [R][256] float4 per block (cr, cg, cb, t).
template <bool CT, bool GUARD, int R>
__device__ __forceinline__ void render_rows_lds_pixels(const float4* __restrict__ planes, int64_t plane_stride,
                                                       const RenderGeom& g, int p_begin, int p_end, int back,
                                                       const float* __restrict__ hv, int x, int y0,
                                                       float4* __restrict__ st) {
    const float fx = (float)x;
    const bool replace_first = !CT || back;
    const int last = p_end - 1;
    auto hom = [&](int p) { return load_hom(hv + (int64_t)(p < last ? p : last) * 9); };
    auto issue = [&](int p, int k, const Hom9& h, TapSet& ts) {
        const int q = p < last ? p : last;
        float px, py;
        render_pos_fast<GUARD>(h.h, fx, (float)(y0 + k), g, px, py);
        issue_taps_padded(make_rsrc(planes + (int64_t)q * plane_stride, g.plane_bytes), g.W, g.H, g.Wp, g.org,
                          g.row, px, py, ts);
    };
    auto consume = [&](const TapSet& ts, int k, bool first) {
        const f32x4 s = blend_taps(ts);
        const float a = first ? 1.0f : s[3];
        const float om = 1.0f - a;
        float4 c = st[k * 256];
        c.x = over(s[0], a, om, c.x);
        c.y = over(s[1], a, om, c.y);
        c.z = over(s[2], a, om, c.z);
        if (CT) c.w = c.w * om;
        st[k * 256] = c;
    };
    TapSet A, B;
    Hom9 h = hom(p_begin), hn = hom(p_begin + 1);
    issue(p_begin, 0, h, A);
    for (int p = p_begin; p < p_end; ++p) {
        const bool first = replace_first && p == p_begin;
#pragma unroll 1
        for (int k = 0; k < R; k += 2) {  // A holds (p, k)
            issue(p, k + 1, h, B);
            __builtin_amdgcn_sched_barrier(0);
            consume(A, k, first);
            if (k + 2 < R)
                issue(p, k + 2, h, A);
            else
                issue(p + 1, 0, hn, A);
            __builtin_amdgcn_sched_barrier(0);
            consume(B, k + 1, first);
        }
        h = hn;
        hn = hom(p + 2);
    }
}

template <bool CT, int R>
__global__ __launch_bounds__(256) void render_rows_lds_kernel(const float4* __restrict__ planes, int64_t plane_stride,
                                                              RenderGeom g, int V, int p_begin, int p_end, int back,
                                                              const float* __restrict__ homs,
                                                              float* __restrict__ out) {
    __shared__ float4 s_state[R * 256];
    constexpr int TY = 4 * R;
    const int tiles_x = (g.W + kTileX - 1) / kTileX;
    const int lb = xcd_logical_block(blockIdx.x, gridDim.x);
    const int v = lb % V;
    const int tile = lb / V;
    const int tx0 = (tile % tiles_x) * kTileX, ty0 = (tile / tiles_x) * TY;
    const int x = tx0 + (int)(threadIdx.x & (kWave - 1));
    const int y0 = ty0 + (int)(threadIdx.x >> 6) * R;
    const float* hv = homs + (int64_t)v * g.P * 9;
    bool ok = true;
    {
        const float x0 = (float)tx0, x1 = (float)min(tx0 + kTileX - 1, g.W - 1);
        const float fy0 = (float)ty0, fy1 = (float)min(ty0 + TY - 1, g.H - 1);
        for (int p = p_begin + (int)threadIdx.x; p < p_end; p += 256)
            ok = ok && div2_rect_safe(hv + (int64_t)p * 9, x0, x1, fy0, fy1);
    }
    const bool proven = __syncthreads_and(ok);
    if (x >= g.W || y0 >= g.H) return;
    float4* st = s_state + threadIdx.x;  // this lane's row k at st[k * 256]
    for (int k = 0; k < R; ++k) st[k * 256] = make_float4(-0.0f, -0.0f, -0.0f, 1.0f);  // plane 0 replaces
    if (proven)
        render_rows_lds_pixels<CT, false, R>(planes, plane_stride, g, p_begin, p_end, back, hv, x, y0, st);
    else
        render_rows_lds_pixels<CT, true, R>(planes, plane_stride, g, p_begin, p_end, back, hv, x, y0, st);
    for (int k = 0; k < R; ++k) {
        const int y = y0 + k;
        if (y >= g.H) break;
        const float4 c = st[k * 256];
        const int64_t o = ((int64_t)v * g.H + y) * g.W + x;
        if (CT) {
            reinterpret_cast<float4*>(out)[o] = c;
        } else {
            out[o * 3 + 0] = c.x;
            out[o * 3 + 1] = c.y;
            out[o * 3 + 2] = c.z;
        }
    }
}

// render_packed_kernel's contract (FAST recipe: H, W >= 2); a 256-thread block = 64 x 4R
// tile, wave w owns rows w*R .. w*R+R-1; XCD-aware (tile, view) order, tile-level
// division proof.
// COUNT (census build, mpiv_render_packed_census): the same kernel also adds up the gather
// instructions its waves issue (the texture path's real work, for bench.py's roofline).
// Rows [y_lo, y_hi) of the frame (the whole frame by default; a row band of a plane-shard
// partial, mpiv_render_packed_ct_rows: the tiles start at y_lo, rows from y_hi on are not stored).
// SAME with R = 6 (the automatic stretched choice) is held to 128 VGPRs, four waves per SIMD: the
// (C, T) flavour needs 129 otherwise (config-5 shard 0.655 vs 0.667 ms; the other R spill there);
// with OOB (135-145 VGPRs) it keeps three
template <bool CT, int R, bool VS = false, bool COUNT = false, int D = 2, bool SAME = false, bool OOB = false>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(SAME && R == 6 && !OOB ? 4 : 1))) void render_rows_kernel(const float4* __restrict__ planes, int64_t plane_stride,
                                                          RenderGeom g, int V, int p_begin, int p_end, int back,
                                                          const float* __restrict__ homs, float* __restrict__ out,
                                                          unsigned long long* __restrict__ census = nullptr,
                                                          int y_lo = 0, int y_hi = -1) {
    constexpr int TY = 4 * R;
    if (y_hi < 0) y_hi = g.H;
    const int tiles_x = (g.W + kTileX - 1) / kTileX;
    const int lb = xcd_logical_block(blockIdx.x, gridDim.x);
    const int v = lb % V;
    const int tile = lb / V;
    const int tx0 = (tile % tiles_x) * kTileX, ty0 = y_lo + (tile / tiles_x) * TY;
    const int x = tx0 + (int)(threadIdx.x & (kWave - 1));
    const int y0 = ty0 + (int)(threadIdx.x >> 6) * R;
    const float* hv = homs + (int64_t)v * g.P * 9;
    bool ok = true, dd = true;
    {
        const float x0 = (float)tx0, x1 = (float)min(tx0 + kTileX - 1, g.W - 1);
        const float fy0 = (float)ty0, fy1 = (float)min(ty0 + TY - 1, g.H - 1);
        for (int p = p_begin + (int)threadIdx.x; p < p_end; p += 256) {
            const float* hp = hv + (int64_t)p * 9;
            const bool safe = div2_rect_safe(hp, x0, x1, fy0, fy1);
            ok = ok && safe;
            dd = dd && safe && tile_dead(hp, x0, x1, fy0, fy1, g);
        }
    }
    const bool proven = __syncthreads_and(ok);
    const bool dead = __syncthreads_and(dd);
    if (x >= g.W || y0 >= y_hi) return;  // rows past y_hi inside [y0, y0+R) are computed, not stored
    float cr[R], cg[R], cb[R], tt[R];
#pragma unroll
    for (int k = 0; k < R; ++k) {
        cr[k] = -0.0f; cg[k] = -0.0f; cb[k] = -0.0f; tt[k] = 1.0f;  // render_packed_pixel: plane 0 replaces
    }
    if (dead) {  // every plane samples the zero border over the whole tile: no positions, no gathers
        composite_zero<CT>(p_begin, p_end, !CT || back, cr[0], cg[0], cb[0], tt[0]);
#pragma unroll
        for (int k = 1; k < R; ++k) {
            cr[k] = cr[0]; cg[k] = cg[0]; cb[k] = cb[0]; tt[k] = tt[0];
        }
    } else if (!proven) {  // rare (w near 0 over the tile): the guarded one-pixel recipe, row by row
        int rows = 0;
        for (int k = 0; k < R && y0 + k < y_hi; ++k, ++rows) {
            const int64_t o = ((int64_t)v * g.H + y0 + k) * g.W + x;
            render_packed_pixel<CT, 1>(planes, plane_stride, g, p_begin, p_end, back, hv, x, y0 + k,
                                       CT ? out + o * 4 : out + o * 3);
        }
        // ~(P + 1) issues of 4 gathers per row (render_packed_pixel's ping-pong)
        if (COUNT && (threadIdx.x & (kWave - 1)) == 0)
            atomicAdd(census, (unsigned long long)rows * 4ull * (unsigned long long)(p_end - p_begin + 1));
        return;
    }
    if (!dead) {
        unsigned nvm = 0;
        if constexpr (VS)
            render_rows_vs_pixels<CT, false, R, D, SAME, OOB>(planes, plane_stride, g, p_begin, p_end, back, hv, x, y0, cr,
                                                         cg, cb, tt, nvm);
        else  // 4 gathers per issue: R per plane plus the first
            render_rows_pixels<CT, false, R>(planes, plane_stride, g, p_begin, p_end, back, hv, x, y0, cr, cg, cb, tt);
        if (!VS) nvm = 4u * (unsigned)(R * (p_end - p_begin) + 1);
        if (COUNT && (threadIdx.x & (kWave - 1)) == 0) atomicAdd(census, (unsigned long long)nvm);
    }
#pragma unroll
    for (int k = 0; k < R; ++k) {
        const int y = y0 + k;
        if (y >= y_hi) break;
        const int64_t o = ((int64_t)v * g.H + y) * g.W + x;
        if (CT) {
            reinterpret_cast<float4*>(out)[o] = make_float4(cr[k], cg[k], cb[k], tt[k]);
        } else {
            out[o * 3 + 0] = cr[k];
            out[o * 3 + 1] = cg[k];
            out[o * 3 + 2] = cb[k];
        }
    }
}

// ---------------------------------------------------------------------------
// two horizontally adjacent pixels per work-item (render_pair_kernel)
// ---------------------------------------------------------------------------
//
// What bounds render_packed_kernel on a camera path is the texture path: four 16-B
// gathers per sample at ~64 B/clk/CU.  Where the sample of pixel x+1 has its north-west
// tap exactly one texel east of pixel x's (floor(px) advanced by one on the same row --
// almost every pair at magnifications near 1), pixel x+1's west taps ARE pixel x's east
// taps, already in registers.  A work-item owns the pair (x, x+1): it always gathers
// pixel x's four taps and pixel x+1's two east taps, and pixel x+1's two west taps only
// when some lane of the wave has a pair that does not share (a wave-uniform branch;
// lanes that share get the buffer's zero range there).  The sharing test compares the
// two tap offsets, so a shared texel is the same memory word: the result is
// bit-identical to the one-pixel kernel.  A wave covers 128 pixels of one row.
constexpr int kPairX = 128;

struct PairTaps {
    f32x4 a0, b0, c0, d0;  // pixel x:   NW, NE, SW, SE
    f32x4 a1, b1, c1, d1;  // pixel x+1: NW (unless shared), NE, SW (unless shared), SE
    float w0[4], w1[4];    // bilinear weights nw, ne, sw, se
    bool share;            // pixel x+1's west taps are pixel x's east taps
};

// floor, weights and the padded-plane byte offset of the north-west tap (issue_taps_padded)
__device__ __forceinline__ int tap_origin(const RenderGeom& g, float px, float py, float* w) {
    const float fx0 = floorf(px), fy0 = floorf(py);
    const float wx = px - fx0, ex = 1.0f - wx;
    const float wy = py - fy0, sy = 1.0f - wy;
    w[0] = sy * ex;
    w[1] = sy * wx;
    w[2] = wy * ex;
    w[3] = wy * wx;
    const int cx = (int)__builtin_amdgcn_fmed3f(fx0, -2.0f, (float)g.W);
    const int cy = (int)__builtin_amdgcn_fmed3f(fy0, -2.0f, (float)g.H);
    return (__mul24(cy, g.Wp) + cx) * 16 + g.org;
}

__device__ __forceinline__ f32x4 blend4w(f32x4 a, f32x4 b, f32x4 c, f32x4 d, const float* w) {
    f32x4 o;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        float acc = a[k] * w[0];
        acc = __builtin_fmaf(b[k], w[1], acc);
        acc = __builtin_fmaf(c[k], w[2], acc);
        acc = __builtin_fmaf(d[k], w[3], acc);
        o[k] = acc;
    }
    return o;
}

template <bool CT, bool GUARD, bool PIPE>
__device__ __forceinline__ void render_pair_pixels(const float4* __restrict__ planes, int64_t plane_stride,
                                                   const RenderGeom& g, int p_begin, int p_end, int back,
                                                   const float* __restrict__ hv, int x, int y, bool second,
                                                   float* __restrict__ out0) {
    const float fx = (float)x, fx1 = (float)(x + 1), fy = (float)y;
    float c0r = -0.0f, c0g = -0.0f, c0b = -0.0f, t0 = 1.0f;  // render_packed_pixel: plane 0 replaces
    float c1r = -0.0f, c1g = -0.0f, c1b = -0.0f, t1 = 1.0f;
    const bool replace_first = !CT || back;
    const int last = p_end - 1;
    auto hom = [&](int p) { return load_hom(hv + (int64_t)(p < last ? p : last) * 9); };
    auto issue = [&](int p, const Hom9& h, PairTaps& ts) {
        const int q = p < last ? p : last;
        float px0, py0, px1, py1;
        render_pos_fast<GUARD>(h.h, fx, fy, g, px0, py0);
        render_pos_fast<GUARD>(h.h, fx1, fy, g, px1, py1);
        const int off0 = tap_origin(g, px0, py0, ts.w0);
        const int off1 = tap_origin(g, px1, py1, ts.w1);
        ts.share = off1 == off0 + 16;
        const __amdgpu_buffer_rsrc_t r = make_rsrc(planes + (int64_t)q * plane_stride, g.plane_bytes);
        if (__builtin_amdgcn_ballot_w64(!ts.share)) {  // wave-uniform: some pair does not share
            const int o = ts.share ? kOOB : off1;
            ts.a1 = llvm_raw_buffer_load_v4f32(r, o, 0, 0);
            ts.c1 = llvm_raw_buffer_load_v4f32(r, o, g.row, 0);
        }
        ts.a0 = llvm_raw_buffer_load_v4f32(r, off0, 0, 0);
        ts.b0 = llvm_raw_buffer_load_v4f32(r, off0 + 16, 0, 0);
        ts.c0 = llvm_raw_buffer_load_v4f32(r, off0, g.row, 0);
        ts.d0 = llvm_raw_buffer_load_v4f32(r, off0 + 16, g.row, 0);
        ts.b1 = llvm_raw_buffer_load_v4f32(r, off1 + 16, 0, 0);
        ts.d1 = llvm_raw_buffer_load_v4f32(r, off1 + 16, g.row, 0);
    };
    auto consume = [&](const PairTaps& ts, bool first) {
        const f32x4 s0 = blend4w(ts.a0, ts.b0, ts.c0, ts.d0, ts.w0);
        const f32x4 a1 = ts.share ? ts.b0 : ts.a1, c1 = ts.share ? ts.d0 : ts.c1;
        const f32x4 s1 = blend4w(a1, ts.b1, c1, ts.d1, ts.w1);
        const float a0 = first ? 1.0f : s0[3], om0 = 1.0f - a0;
        const float aa1 = first ? 1.0f : s1[3], om1 = 1.0f - aa1;
        c0r = over(s0[0], a0, om0, c0r);
        c0g = over(s0[1], a0, om0, c0g);
        c0b = over(s0[2], a0, om0, c0b);
        c1r = over(s1[0], aa1, om1, c1r);
        c1g = over(s1[1], aa1, om1, c1g);
        c1b = over(s1[2], aa1, om1, c1b);
        if (CT) {
            t0 = t0 * om0;
            t1 = t1 * om1;
        }
    };
    if (PIPE) {  // two planes' taps in flight (117 VGPRs: 4 waves/SIMD)
        PairTaps A, B;
        Hom9 hA = hom(p_begin), hB = hom(p_begin + 1);
        issue(p_begin, hA, A);
        hA = hom(p_begin + 2);
        int p = p_begin;
        for (; p + 1 < p_end; p += 2) {  // A holds plane p, B will hold p + 1
            issue(p + 1, hB, B);
            hB = hom(p + 3);
            __builtin_amdgcn_sched_barrier(0);
            consume(A, replace_first && p == p_begin);
            issue(p + 2, hA, A);
            hA = hom(p + 4);
            __builtin_amdgcn_sched_barrier(0);
            consume(B, false);
        }
        if (p < p_end) consume(A, replace_first && p == p_begin);
    } else {  // one plane in flight per work-item, i.e. two pixels' worth (twice the waves)
        PairTaps A;
        Hom9 h = hom(p_begin);
        for (int p = p_begin; p < p_end; ++p) {
            issue(p, h, A);
            h = hom(p + 1);
            consume(A, replace_first && p == p_begin);
        }
    }
    if (CT) {
        float4* o = reinterpret_cast<float4*>(out0);
        o[0] = make_float4(c0r, c0g, c0b, t0);
        if (second) o[1] = make_float4(c1r, c1g, c1b, t1);
    } else {
        out0[0] = c0r;
        out0[1] = c0g;
        out0[2] = c0b;
        if (second) {
            out0[3] = c1r;
            out0[4] = c1g;
            out0[5] = c1b;
        }
    }
}

// render_packed_kernel's contract (FAST recipe: H, W >= 2); 256 threads = 4 rows x 128
// pixels, XCD-aware (tile, view) order, tile-level division proof.
template <bool CT, bool PIPE>
__global__ __launch_bounds__(256) void render_pair_kernel(const float4* __restrict__ planes, int64_t plane_stride,
                                                          RenderGeom g, int V, int p_begin, int p_end, int back,
                                                          const float* __restrict__ homs, float* __restrict__ out) {
    const int tiles_x = (g.W + kPairX - 1) / kPairX;
    const int lb = xcd_logical_block(blockIdx.x, gridDim.x);
    const int v = lb % V;
    const int tile = lb / V;
    const int tx0 = (tile % tiles_x) * kPairX, ty0 = (tile / tiles_x) * kTileY;
    const int x = tx0 + 2 * (threadIdx.x & (kWave - 1));
    const int y = ty0 + (threadIdx.x >> 6);
    const float* hv = homs + (int64_t)v * g.P * 9;
    bool ok = true;
    {
        const float x0 = (float)tx0, x1 = (float)min(tx0 + kPairX - 1, g.W - 1);
        const float y0 = (float)ty0, y1 = (float)min(ty0 + kTileY - 1, g.H - 1);
        for (int p = p_begin + (int)threadIdx.x; p < p_end; p += 256)
            ok = ok && div2_rect_safe(hv + (int64_t)p * 9, x0, x1, y0, y1);
    }
    const bool proven = __syncthreads_and(ok);
    if (x >= g.W || y >= g.H) return;
    const int64_t o = ((int64_t)v * g.H + y) * g.W + x;
    float* out0 = CT ? out + o * 4 : out + o * 3;
    const bool second = x + 1 < g.W;
    if (proven) {
        render_pair_pixels<CT, false, PIPE>(planes, plane_stride, g, p_begin, p_end, back, hv, x, y, second, out0);
    } else {  // rare (w near 0 over the tile): the guarded one-pixel recipe, pixel by pixel
        render_packed_pixel<CT, 1>(planes, plane_stride, g, p_begin, p_end, back, hv, x, y, out0);
        if (second)
            render_packed_pixel<CT, 1>(planes, plane_stride, g, p_begin, p_end, back, hv, x + 1, y,
                                       out0 + (CT ? 4 : 3));
    }
}

// ---------------------------------------------------------------------------
// native [B,H,W,P,C=4] layout, arbitrary element strides
// ---------------------------------------------------------------------------

struct NativeStrides {
    int64_t b, y, x, p, c;
};

// One RGBA texel of the native layout.  The address is always clamped into the image
// (so it is valid memory) and the value is zeroed when the tap is outside it --
// grid_sample's zeros padding.  VEC: channels contiguous and 16-B aligned texels.
template <bool VEC>
__device__ __forceinline__ f32x4 ld_texel(const float* __restrict__ plane, const NativeStrides& s, int W, int H,
                                          int ix, int iy, bool ok) {
    const int cx = ix < 0 ? 0 : (ix >= W ? W - 1 : ix);
    const int cy = iy < 0 ? 0 : (iy >= H ? H - 1 : iy);
    const float* t = plane + (int64_t)cy * s.y + (int64_t)cx * s.x;
    f32x4 v;
    if (VEC) {
        v = *reinterpret_cast<const f32x4*>(t);
    } else {
        v[0] = t[0]; v[1] = t[s.c]; v[2] = t[2 * s.c]; v[3] = t[3 * s.c];
    }
    const f32x4 z = {0.f, 0.f, 0.f, 0.f};
    return ok ? v : z;
}

// The reference's own [B,H,W,P,4] tensor, read in place (no pack).  Same per-plane
// arithmetic as the packed kernel; texel gathers stride over the P*16-B pixel rows.
template <bool VEC, bool FAST>
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
    float cr = -0.0f, cg = -0.0f, cb = -0.0f;  // see render_packed_kernel: plane 0 replaces
    for (int p = 0; p < g.P; ++p) {
        float px, py;
        render_pos<FAST>(hv + (int64_t)p * 9, fx, fy, g, px, py);
        const Bilinear b = bilinear_setup(px, py, g.W, g.H);
        const float* pl = img + (int64_t)p * s.p;
        TapSet t;
        t.nw = b.nw; t.ne = b.ne; t.sw = b.sw; t.se = b.se;
        t.a = ld_texel<VEC>(pl, s, g.W, g.H, b.ix, b.iy, b.x0 && b.y0);
        t.b = ld_texel<VEC>(pl, s, g.W, g.H, b.ix + 1, b.iy, b.x1 && b.y0);
        t.c = ld_texel<VEC>(pl, s, g.W, g.H, b.ix, b.iy + 1, b.x0 && b.y1);
        t.d = ld_texel<VEC>(pl, s, g.W, g.H, b.ix + 1, b.iy + 1, b.x1 && b.y1);
        const f32x4 c = blend_taps(t);
        const float a = p == 0 ? 1.0f : c[3];
        const float om = 1.0f - a;
        cr = over(c[0], a, om, cr);
        cg = over(c[1], a, om, cg);
        cb = over(c[2], a, om, cb);
    }
    const int64_t o = (((int64_t)v * g.H + y) * g.W + x) * 3;
    out[o + 0] = cr;
    out[o + 1] = cg;
    out[o + 2] = cb;
}

// ---------------------------------------------------------------------------
// layout pack: one view of [H,W,P,C=4] (any strides) -> [P][H+4][W+4] float4 with a
// 2-texel zero border.  A block moves 64 padded pixels x 16 planes through LDS so both
// sides are coalesced: reads are 16 planes x 16 B = 256 B per pixel, writes 64 pixels
// x 16 B = 1 KiB per plane; border pixels are written as zeros.
// ---------------------------------------------------------------------------

constexpr int kPackPix = 64;
constexpr int kPackPl = 16;

__global__ __launch_bounds__(256) void pack_planes_kernel(const float* __restrict__ mpi, NativeStrides s,
                                                          int H, int W, int P, FastDiv wp_div,
                                                          float4* __restrict__ packed, int64_t plane_stride) {
    __shared__ float4 tile[kPackPl][kPackPix + 1];
    const int64_t npix = plane_stride;  // (H+4)*(W+4) < 2^27
    const int64_t pix0 = (int64_t)blockIdx.x * kPackPix;
    const int p0 = blockIdx.y * kPackPl;
    // load: thread -> (pixel i, plane j), plane fastest
    for (int k = threadIdx.x; k < kPackPix * kPackPl; k += blockDim.x) {
        const int j = k % kPackPl, i = k / kPackPl;
        const int64_t pix = pix0 + i;
        const int p = p0 + j;
        float4 val = make_float4(0.f, 0.f, 0.f, 0.f);
        if (pix < npix && p < P) {
            const int yp = (int)fast_div((unsigned)pix, wp_div);
            const int yy = yp - kPad, xx = (int)pix - yp * (int)wp_div.d - kPad;
            if ((unsigned)yy < (unsigned)H && (unsigned)xx < (unsigned)W) {
                const float* src = mpi + (int64_t)yy * s.y + (int64_t)xx * s.x + (int64_t)p * s.p;
                if (s.c == 1 && ((reinterpret_cast<uintptr_t>(src) & 15) == 0)) {
                    val = *reinterpret_cast<const float4*>(src);
                } else {
                    val = make_float4(src[0], src[s.c], src[2 * s.c], src[3 * s.c]);
                }
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
