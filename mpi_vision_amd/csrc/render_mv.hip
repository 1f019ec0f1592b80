// render_mv.hip -- multi-view fused warp + over-composite with the planes' source
// footprints staged through LDS: the mpiv_render_packed kernel when a launch renders
// several views of one MPI (a camera path, a broadcast batch).
//
// Why it exists: the direct kernel (render.hip) gathers four 16-B taps per plane-pixel
// through the vector L1 and keeps the texture path ~87 % busy (PMC, config 4).  The views
// of a camera path see almost the same source footprint per output tile, so one block
// here renders one 64x4 output tile for kMVB consecutive views: per plane it stages the
// UNION of those views' footprints in LDS once (one coalesced fill, ~1/15 of the direct
// kernel's L1 bytes; texture-path busy drops to ~14 %) and every view's taps become
// ds_read_b128s.  The per-sample recipe is render.hip's, so the output is bit-identical.
// Measured (MI355X, config 4, 125 views per launch): 30.5 ms against the direct kernel's
// 30.4 ms -- relieving the texture path exposes the VALU issue of the recipe (~94 VALU
// per sample here vs 81 direct, 68 % VALU busy), so this is an opt-in A/B variant
// (MPIV_RENDER_MV=1), not the default; DESIGN.md §4.
//
// Per block (256 threads = 4 waves; one 64-pixel output row per wave):
//  1. prologue: every (plane, view, tile corner) triple goes through the exact
//     per-pixel recipe; plane p's box is [floor(min px) - 1, floor(max px) + 2] x (the
//     same in y) over all views and corners, clipped to the padded planes' [-2, W+1] x
//     [-2, H+1].  While w keeps its sign over the tile, the exact image of the tile is
//     the convex hull of its corners' images and rounded interior positions stay within
//     a texel of the corner box, which the margin covers (render_lds.hip).  Planes whose
//     w changes sign, whose positions are non-finite or huge, or whose box does not fit
//     the staging buffer are gathered from global memory for the whole tile.
//  2. planes back to front with two LDS buffers: plane p+1's footprint is loaded into
//     registers while plane p is composited for all views, then written to the other
//     buffer; one barrier per plane.  The fill's latency hides behind kMVB views of
//     work.  A sample whose tap origin is nevertheless not staged (image borders,
//     rounding at ill-conditioned geometry, NaN) is gathered from global memory
//     (lds_sample), so the result never depends on the box being right.
#include "mpiv_common.hpp"

namespace mpiv {

constexpr int kMTX = 64;                   // tile width (one wave = one output row)
constexpr int kMTY = 4;                    // tile height (4 waves)
constexpr int kMThreads = kMTX * kMTY;
constexpr int kMVB = 8;                    // views per block
constexpr int kMI = 4 * kMVB;              // box items (view, corner) per plane
constexpr int kMCap = 1024;                // texels per staging buffer (16 KiB)
constexpr int kMFill = kMCap / kMThreads;  // staged texels per thread per plane
constexpr int kMMaxP = 256;                // planes per launch in the box table
constexpr int kMMaxPitch = 256;            // footprints wider than this go direct
constexpr int kMMinViews = 4;              // fewer views per launch: render.hip
constexpr int kMG = 2;                     // views whose samples are in flight together

// shrink > 0 narrows every box by that many texels per side (tests: forces the
// per-sample global fallback); 0 in production.
template <bool CT>
__global__ __launch_bounds__(kMThreads) void render_mv_kernel(const float4* __restrict__ planes,
                                                              int64_t plane_stride, RenderGeom g, int V,
                                                              int p_begin, int p_end, int back, int shrink,
                                                              const float* __restrict__ homs,
                                                              float* __restrict__ out) {
    __shared__ __attribute__((aligned(16))) float4 s_tex[2][kMCap];
    __shared__ int4 s_box[kMMaxP];  // per plane: x_lo, y_lo, rows, staged (1) / direct (0)
    __shared__ int s_pitch;
    // the block's views' homographies of the plane in flight, double-buffered with the
    // texels (12-float rows: 16-B aligned ds_read_b128s).  Read from LDS they are counted
    // by lgkmcnt in order with the tap reads; as scalar loads each view's s_load would
    // drain every outstanding LDS read (SMEM returns out of order: lgkmcnt(0)).
    __shared__ __attribute__((aligned(16))) float s_hom[2][kMVB][12];

    const int tiles_x = (g.W + kMTX - 1) / kMTX;
    const int ngroups = (V + kMVB - 1) / kMVB;
    const int lb = xcd_logical_block(blockIdx.x, gridDim.x);
    const int vg0 = (lb % ngroups) * kMVB;  // first view of this block
    const int nv = min(kMVB, V - vg0);      // views of this block (block-uniform)
    const int tile = lb / ngroups;
    const int tx0 = (tile % tiles_x) * kMTX, ty0 = (tile / tiles_x) * kMTY;
    const int x = tx0 + (threadIdx.x & (kWave - 1)), y = ty0 + (threadIdx.x >> 6);
    const bool active = x < g.W && y < g.H;
    const int np = p_end - p_begin;

    if (threadIdx.x == 0) s_pitch = 0;
    __syncthreads();

    // ---- 1. footprint boxes: item q -> (plane q/kMI, view (q/4)%kMVB, corner q%4); the
    // kMI items of one plane are consecutive lanes, reduced with xor shuffles
    static_assert(kMI <= kWave && (kMI & (kMI - 1)) == 0, "one plane's box items must fit a wave");
    const int cx1 = min(tx0 + kMTX - 1, g.W - 1), cy1 = min(ty0 + kMTY - 1, g.H - 1);
    for (int q0 = 0; q0 < kMI * np; q0 += kMThreads) {
        const int q = q0 + threadIdx.x;
        const bool live = q < kMI * np;  // uniform per kMI-lane group
        const int pl = p_begin + (live ? q / kMI : 0);
        const int corner = q & 3;
        const int v = min(vg0 + ((q >> 2) & (kMVB - 1)), V - 1);
        const float fx = (float)((corner & 1) ? cx1 : tx0), fy = (float)((corner & 2) ? cy1 : ty0);
        const float* h = homs + ((int64_t)v * g.P + pl) * 9;
        float px, py;
        render_pos<true>(h, fx, fy, g, px, py);
        float w = __builtin_fmaf(h[7], fy, h[6] * fx) + h[8];
        w = (w == 0.0f) ? w + 1e-8f : w;
        const bool fin = __builtin_isfinite(px) && __builtin_isfinite(py) && __builtin_fabsf(px) < 1e7f &&
                         __builtin_fabsf(py) < 1e7f;
        float xmin = floorf(px), xmax = xmin, ymin = floorf(py), ymax = ymin;
        int pos = fin && w > 0.0f, neg = fin && w < 0.0f;
#pragma unroll
        for (int m = 1; m < kMI; m <<= 1) {
            xmin = fminf(xmin, __shfl_xor(xmin, m));
            xmax = fmaxf(xmax, __shfl_xor(xmax, m));
            ymin = fminf(ymin, __shfl_xor(ymin, m));
            ymax = fmaxf(ymax, __shfl_xor(ymax, m));
            pos &= __shfl_xor(pos, m);
            neg &= __shfl_xor(neg, m);
        }
        if (live && (q & (kMI - 1)) == 0) {
            const bool ok = pos || neg;
            const int xl = ok ? max((int)xmin - 1 + shrink, -2) : 0;
            const int xh = ok ? min((int)xmax + 2 - shrink, g.W + 1) : 0;
            const int yl = ok ? max((int)ymin - 1 + shrink, -2) : 0;
            const int yh = ok ? min((int)ymax + 2 - shrink, g.H + 1) : 0;
            const int width = xh - xl + 1, rows = yh - yl + 1;
            const bool staged = ok && width >= 2 && rows >= 2 && width <= kMMaxPitch && rows <= kMCap &&
                                width * rows <= kMCap;
            s_box[q / kMI] = make_int4(xl, yl, rows, staged ? 1 : 0);
            if (staged) atomicMax(&s_pitch, width);
        }
    }
    __syncthreads();
    const int pitch = __builtin_amdgcn_readfirstlane(s_pitch);  // common row pitch of the staged boxes

    // this thread's share of a footprint: texels idx = tid + 256*k, as offsets (in
    // texels) from the box origin in the padded plane
    int rel[kMFill];
#pragma unroll
    for (int k = 0; k < kMFill; ++k) {
        const int idx = threadIdx.x + kMThreads * k;
        const int row = pitch > 0 ? idx / pitch : 0;
        rel[k] = row * g.Wp + (idx - row * pitch);
    }
    auto load_box = [&](int i) {
        const int4 b = s_box[i];
        return make_int4(__builtin_amdgcn_readfirstlane(b.x), __builtin_amdgcn_readfirstlane(b.y),
                         __builtin_amdgcn_readfirstlane(b.z), __builtin_amdgcn_readfirstlane(b.w));
    };
    auto staged = [&](const int4& b) { return b.w != 0 && b.z * pitch <= kMCap; };

    // register staging (render_lds.hip says why not LDS-DMA); texels past the box are
    // loaded too (real memory or the buffer's zero range) and never read
    f32x4 stg[kMFill];
    float hstg = 0.0f;  // thread t < 9*kMVB stages homography element t of the next plane
    const int hj = threadIdx.x / 9, he = threadIdx.x - 9 * (threadIdx.x / 9);
    const bool hthread = threadIdx.x < 9 * kMVB;
    const float* hsrc = homs + ((int64_t)min(vg0 + hj, V - 1) * g.P) * 9 + he;
    auto fetch_hom = [&](int pl) {
        if (hthread) hstg = hsrc[(int64_t)pl * 9];
    };
    auto commit_hom = [&](int buf) {
        if (hthread) s_hom[buf][hj][he] = hstg;
    };
    auto fetch = [&](int pl, const int4& bx) {
        const __amdgpu_buffer_rsrc_t r = make_rsrc(planes + (int64_t)pl * plane_stride, g.plane_bytes);
        const int box_org = (bx.y + kPad) * g.Wp + bx.x + kPad;  // >= 0: boxes start at -2
        const int nfp = bx.z * pitch;
#pragma unroll
        for (int k = 0; k < kMFill; ++k)
            if (kMThreads * k < nfp) stg[k] = llvm_raw_buffer_load_v4f32(r, (box_org + rel[k]) * 16, 0, 0);
    };
    auto commit = [&](int buf, const int4& bx) {
        const int nfp = bx.z * pitch;
#pragma unroll
        for (int k = 0; k < kMFill; ++k)
            if (kMThreads * k < nfp) *reinterpret_cast<f32x4*>(&s_tex[buf][threadIdx.x + kMThreads * k]) = stg[k];
    };

    const float fx = (float)x, fy = (float)y;
    float cr[kMVB], cg[kMVB], cb[kMVB], tt[kMVB];
#pragma unroll
    for (int j = 0; j < kMVB; ++j) {
        cr[j] = -0.0f;  // plane p_begin replaces it exactly (render.hip)
        cg[j] = -0.0f;
        cb[j] = -0.0f;
        tt[j] = 1.0f;
    }
    const bool replace_first = !CT || back;
    auto consume = [&](int j, const f32x4& s, bool first) {
        const float a = first ? 1.0f : s[3];
        const float om = 1.0f - a;
        cr[j] = over(s[0], a, om, cr[j]);
        cg[j] = over(s[1], a, om, cg[j]);
        cb[j] = over(s[2], a, om, cb[j]);
        if (CT) tt[j] = tt[j] * om;
    };

    int4 bx_next = load_box(0);
    fetch_hom(p_begin);
    if (staged(bx_next)) {
        fetch(p_begin, bx_next);
        commit(0, bx_next);
    }
    commit_hom(0);
    __syncthreads();
    for (int p = p_begin; p < p_end; ++p) {
        const int buf = (p - p_begin) & 1;
        const int4 bx = bx_next;
        const bool more = p + 1 < p_end;
        if (more) {
            bx_next = load_box(p + 1 - p_begin);
            fetch_hom(p + 1);
            if (staged(bx_next)) fetch(p + 1, bx_next);
        }
        const bool first = replace_first && p == p_begin;
        if (active) {
            const __amdgpu_buffer_rsrc_t r = make_rsrc(planes + (int64_t)p * plane_stride, g.plane_bytes);
            if (staged(bx)) {
                const LdsBox lbx = make_lds_box(bx.x, bx.y, bx.z, pitch, g.W, g.H);
                const float4* tex = s_tex[buf];
                // kMG views at a time, phase by phase (positions, tap reads, blends), with
                // the rare fix-ups behind wave-uniform tests: their LDS reads are in flight
                // together instead of one round trip per view
#pragma unroll
                for (int j0 = 0; j0 < kMVB; j0 += kMG) {
                    if (j0 < nv) {
                        float qu[kMG], qv[kMG];
                        bool fast = true;
#pragma unroll
                        for (int jj = 0; jj < kMG; ++jj) {
                            const float* h = s_hom[buf][j0 + jj];
                            const float u = __builtin_fmaf(h[1], fy, h[0] * fx) + h[2];
                            const float v = __builtin_fmaf(h[4], fy, h[3] * fx) + h[5];
                            const float w = __builtin_fmaf(h[7], fy, h[6] * fx) + h[8];
                            fast = fast && div2_safe(u, v, w);
                            div2_fast(u, v, w, qu[jj], qv[jj]);
                        }
                        if (__builtin_amdgcn_ballot_w64(!fast)) {  // rare: divide_safe2's slow path
#pragma unroll
                            for (int jj = 0; jj < kMG; ++jj) {
                                const float* h = s_hom[buf][j0 + jj];
                                const float u = __builtin_fmaf(h[1], fy, h[0] * fx) + h[2];
                                const float v = __builtin_fmaf(h[4], fy, h[3] * fx) + h[5];
                                const float w = __builtin_fmaf(h[7], fy, h[6] * fx) + h[8];
                                if (!div2_safe(u, v, w)) divide_safe2(u, v, w, qu[jj], qv[jj]);
                            }
                        }
                        float px[kMG], py[kMG];
                        TapSet ts[kMG];
                        bool ok = true;
#pragma unroll
                        for (int jj = 0; jj < kMG; ++jj) {
                            const float cx = div_const(qu[jj], g.hm1, g.rc_hm1);  // SWAPPED x / (H-1), utils.py:188
                            const float cy = div_const(qv[jj], g.wm1, g.rc_wm1);  //         y / (W-1)
                            px[jj] = unnormalize(to_grid(cx), g.half_w);
                            py[jj] = unnormalize(to_grid(cy), g.half_h);
                            ok = lds_issue(tex, lbx, px[jj], py[jj], ts[jj]) && ok;
                        }
                        f32x4 sm[kMG];
#pragma unroll
                        for (int jj = 0; jj < kMG; ++jj) sm[jj] = blend_taps(ts[jj]);
                        if (__builtin_amdgcn_ballot_w64(!ok)) {  // wave-uniform test, then per lane
                            if (!ok) {                           // a tap origin not staged: global gather
#pragma unroll
                                for (int jj = 0; jj < kMG; ++jj)
                                    issue_taps_padded(r, g.W, g.H, g.Wp, g.org, g.row, px[jj], py[jj], ts[jj]);
#pragma unroll
                                for (int jj = 0; jj < kMG; ++jj) sm[jj] = blend_taps(ts[jj]);
                            }
                        }
#pragma unroll
                        for (int jj = 0; jj < kMG; ++jj)
                            if (j0 + jj < nv) consume(j0 + jj, sm[jj], first);
                    }
                }
            } else {
#pragma unroll
                for (int j = 0; j < kMVB; ++j) {
                    if (j < nv) {
                        float px, py;
                        render_pos<true>(s_hom[buf][j], fx, fy, g, px, py);
                        TapSet ts;
                        issue_taps_padded(r, g.W, g.H, g.Wp, g.org, g.row, px, py, ts);
                        consume(j, blend_taps(ts), first);
                    }
                }
            }
        }
        if (more) {
            if (staged(bx_next)) commit(buf ^ 1, bx_next);
            commit_hom(buf ^ 1);
        }
        __syncthreads();
    }
    if (!active) return;
#pragma unroll
    for (int j = 0; j < kMVB; ++j) {
        if (j < nv) {
            const int64_t o = ((int64_t)(vg0 + j) * g.H + y) * g.W + x;
            if (CT) {
                reinterpret_cast<float4*>(out)[o] = make_float4(cr[j], cg[j], cb[j], tt[j]);
            } else {
                out[o * 3 + 0] = cr[j];
                out[o * 3 + 1] = cg[j];
                out[o * 3 + 2] = cb[j];
            }
        }
    }
}

}  // namespace mpiv
