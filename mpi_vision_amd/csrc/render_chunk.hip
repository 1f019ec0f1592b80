// render_chunk.hip -- mpi_render_view_torch (utils.py:267-294) reading the reference's
// own [B,H,W,P,4] tensor IN PLACE at the packed kernel's coalescing, so the training
// caller (non-broadcast MPI per view, ipynb cell 12 L42) pays no per-view pack.
//
// In that layout the P texels of one pixel are one contiguous P*16-B run, so a plane's
// texels are P*16 B apart: render_native_kernel's one-pixel-per-lane gathers touch one
// 128-B line per 16-B tap.  Here the lanes of a wave are (pixel, plane-in-chunk) pairs:
// with CH planes per chunk, lane l samples plane  c*CH + l%CH  of pixel  l/CH  (+ the
// sub-step's pixel base), so the CH lanes of one pixel read CH consecutive texels of one
// pixel run -- a whole 128-B line for CH = 8 -- and one tap instruction covers 64/CH
// pixels x CH planes, the same 1 KiB in 8 lines as a packed-layout wave row.
//
// Compositing must stay sequential per pixel (the unfused over-operator rounds in the
// reference's order, back to front), so the blended samples go through a per-wave LDS
// slot: after the CH sub-steps of a chunk the slot holds 64 pixels x CH planes, and lane
// l re-reads pixel l's CH samples (one ds_read_b128 each) and composites them in order.
// Slot rows are XOR-swizzled so both the sub-step writes and the per-pixel reads are
// bank-conflict free.  The per-sample arithmetic is render_packed_kernel's recipe
// (tile-level division proof, exact constant divisions, ATen weights, 4-tap fma chain),
// so the output is bit-identical to the other render kernels; grid_sample's zero
// padding is per tap: an out-of-image tap gets the buffer's out-of-range offset.
#include "mpiv_common.hpp"

namespace mpiv {

// one sample position of render_packed_kernel's recipe for an arbitrary (per-lane) plane
// homography held in VGPRs
template <bool GUARD>
__device__ __forceinline__ void chunk_pos(const float* h, float fx, float fy, const RenderGeom& g, float& px,
                                          float& py) {
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

struct ChunkGeom {
    int row_t, pix_t;  // texel (16-B) strides of a row and a pixel in the reference tensor
    int rec_bytes;     // buffer range from a chunk's base: every live tap is below it
};

// One sample in flight: four taps + the fractional offsets; the bilinear weights are
// formed when the taps are blended (the same products as issue_taps_padded's, so the
// result is identical) -- two VGPRs fewer per sample in flight.
struct ChunkTaps {
    f32x4 a, b, c, d;  // NW, NE, SW, SE
    float wx, wy;
};

__device__ __forceinline__ f32x4 blend_chunk(const ChunkTaps& t) {
    const float ex = 1.0f - t.wx, sy = 1.0f - t.wy;
    const float nw = sy * ex, ne = sy * t.wx, sw = t.wy * ex, se = t.wy * t.wx;
    f32x4 o;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        float acc = t.a[k] * nw;
        acc = __builtin_fmaf(t.b[k], ne, acc);
        acc = __builtin_fmaf(t.c[k], sw, acc);
        acc = __builtin_fmaf(t.d[k], se, acc);
        o[k] = acc;
    }
    return o;
}

// Issue the four taps of one (pixel, plane) sample from the in-place tensor.  Tap origin
// clamped into [-2, W] x [-2, H] (defined int conversion; NaN maps to a bound and its NaN
// weights still poison the sample, as in the reference); a tap outside the image, or any
// tap of a lane past the last plane, gets kOOB: the buffer unit returns 0 without an access.
// Returns the number of taps inside the image (0 for dead lanes; the backward counts the
// texel contributions it must find, render_bwd.hip).
__device__ __forceinline__ int issue_taps_chunk(__amdgpu_buffer_rsrc_t r, const RenderGeom& g, const ChunkGeom& cg,
                                                int jt, bool live, float px, float py, ChunkTaps& t) {
    const float fx0 = floorf(px), fy0 = floorf(py);
    t.wx = px - fx0;
    t.wy = py - fy0;
    const int ix = (int)__builtin_amdgcn_fmed3f(fx0, -2.0f, (float)g.W);
    const int iy = (int)__builtin_amdgcn_fmed3f(fy0, -2.0f, (float)g.H);
    const bool x0 = (unsigned)ix < (unsigned)g.W, x1 = (unsigned)(ix + 1) < (unsigned)g.W;
    const bool y0 = live && (unsigned)iy < (unsigned)g.H, y1 = live && (unsigned)(iy + 1) < (unsigned)g.H;
    // wrapping 32-bit arithmetic: the value is only used where every tap index is valid
    const int off = (int)(((unsigned)__mul24(iy, cg.row_t) + (unsigned)__mul24(ix, cg.pix_t) + (unsigned)jt) * 16u);
    const int pb = cg.pix_t * 16, rb = cg.row_t * 16;
    t.a = llvm_raw_buffer_load_v4f32(r, (x0 && y0) ? off : kOOB, 0, 0);
    t.b = llvm_raw_buffer_load_v4f32(r, (x1 && y0) ? off + pb : kOOB, 0, 0);
    t.c = llvm_raw_buffer_load_v4f32(r, (x0 && y1) ? off + rb : kOOB, 0, 0);
    t.d = llvm_raw_buffer_load_v4f32(r, (x1 && y1) ? off + rb + pb : kOOB, 0, 0);
    return ((int)x0 + (int)x1) * ((int)y0 + (int)y1);
}

// LDS: [4 waves][64 / SPLIT pixels][CH + 1] float4 sample slots (one pad texel per pixel
// row), then the view's P homographies (9 floats each).  The pad makes both access shapes
// bank-conflict free with IMMEDIATE offsets: a sub-step's ds_write_b128 covers CH
// contiguous texels per pixel row, and the composite's per-plane ds_read_b128 has its 16
// lanes of an LDS cycle on rows (CH+1)*16 B apart = 16 distinct four-bank groups
// (MI355X_MICROARCH.md §LDS; checked for CH = 4 and 8).
template <int CH, int SPLIT>
constexpr int chunk_slot_floats() {
    return 4 * (kWave / SPLIT) * (CH + 1) * 4;
}

// R rows per wave (R > 1: SPLIT == 1): the wave renders rows y0 .. y0+R-1 of its 64 columns
// with the chunk loop OUTSIDE the row loop, so row r+1's north taps are the texels row r
// gathered moments before (L1/L2 hits instead of HBM re-reads: a 64 x 4R block tile re-reads
// only its outer halo).  The A/B tap pipeline runs on across rows and chunks.  Rows past the
// frame (nrows < R, wave-uniform) re-sample the last row and are neither composited nor
// stored.
template <int CH, int SPLIT, int R, bool GUARD>
__device__ __forceinline__ void render_chunk_wave(const float* __restrict__ view, const RenderGeom& g,
                                                  const ChunkGeom& cg, const float* __restrict__ hs,
                                                  f32x4* __restrict__ slot, int tx0, int y0, int nrows_, int lane,
                                                  float (&cr)[R], float (&cg_)[R], float (&cb)[R],
                                                  float4* __restrict__ ck, int64_t ck_stride) {
    static_assert(R == 1 || SPLIT == 1, "R rows per wave composite whole chunks");
    constexpr int PPS = kWave / CH;  // pixels per sub-step
    const int nrows = R == 1 ? 1 : nrows_;  // wave-uniform
    const int j = lane % CH, i = lane / CH;
    const int nchunk = (g.P + CH - 1) / CH;
    float h[9];
    auto load_h = [&](int c, float* d) {
        const int p = min(c * CH + j, g.P - 1);
#pragma unroll
        for (int k = 0; k < 9; ++k) d[k] = hs[p * 9 + k];
    };
    auto rsrc = [&](int c) {
        return make_rsrc(view + (int64_t)c * CH * 4, cg.rec_bytes);
    };
    // sub-step k of row r, chunk c: pixel (tx0 + k*PPS + i, row r), plane c*CH + j
    auto issue = [&](int c, int r, int k, const float* hh, ChunkTaps& ts) {
        float px, py;
        const float fy = (float)(y0 + min(r, nrows - 1));
        chunk_pos<GUARD>(hh, (float)(tx0 + k * PPS + i), fy, g, px, py);
        issue_taps_chunk(rsrc(c), g, cg, j, c * CH + j < g.P, px, py, ts);
    };
    constexpr int QP = kWave / SPLIT;  // pixels per composite phase
    constexpr int KP = CH / SPLIT;     // sub-steps per composite phase
    auto put = [&](int k, const ChunkTaps& ts) { slot[((k * PPS + i) % QP) * (CH + 1) + j] = blend_chunk(ts); };
    // composite phase h of row r: lane = pixel tx0 + lane (lanes of that phase only), planes
    // c*CH .. c*CH+CH-1 back to front
    auto composite = [&](int c, int hph, int r) {
        auto over_px = [&](const f32x4& s, bool first) {
            const float a = first ? 1.0f : s[3];  // plane 0 replaces (render_packed_pixel)
            const float om = 1.0f - a;
            cr[r] = over(s[0], a, om, cr[r]);
            cg_[r] = over(s[1], a, om, cg_[r]);
            cb[r] = over(s[2], a, om, cb[r]);
        };
        if (SPLIT == 1 || lane / QP == hph) {
            const f32x4* row = slot + (lane % QP) * (CH + 1);
            if (c * CH + CH <= g.P) {  // full chunk: reads in flight 4 at a time, no branches
#pragma unroll
                for (int j0 = 0; j0 < CH; j0 += 4) {
                    f32x4 s[4];
#pragma unroll
                    for (int jj = 0; jj < 4; ++jj) s[jj] = row[j0 + jj];
#pragma unroll
                    for (int jj = 0; jj < 4; ++jj) over_px(s[jj], c == 0 && j0 + jj == 0);
                }
            } else {
                for (int jj = 0; c * CH + jj < g.P; ++jj) over_px(row[jj], c * CH + jj == 0);
            }
        }
    };
    ChunkTaps A, B;
    load_h(0, h);
    issue(0, 0, 0, h, A);
    for (int c = 0; c < nchunk; ++c) {
        const int cn = c + 1 < nchunk ? c + 1 : c;  // past the end: re-issue (cached, unused)
        // training: the colour before chunk c, the render backward's checkpoint (render_bwd.hip)
        if (ck && c > 0) {
#pragma unroll
            for (int r = 0; r < R; ++r)
                if (r < nrows) ck[c * ck_stride + (int64_t)r * g.W] = make_float4(cr[r], cg_[r], cb[r], 0.0f);
        }
#pragma unroll
        for (int r = 0; r < R; ++r) {
#pragma unroll
            for (int k = 0; k < CH; k += 2) {  // A holds sub-step k of row r
                issue(c, r, k + 1, h, B);
                __builtin_amdgcn_sched_barrier(0);
                put(k, A);
                if (k + 2 < CH) {
                    issue(c, r, k + 2, h, A);
                } else if (r + 1 < R) {
                    issue(c, r + 1, 0, h, A);
                } else {
                    load_h(cn, h);  // the next chunk's homography (LDS) replaces this one's
                    issue(cn, 0, 0, h, A);
                }
                __builtin_amdgcn_sched_barrier(0);
                put(k + 1, B);
                if ((k + 2) % KP == 0 && r < nrows) composite(c, (k + 1) / KP, r);
                if (R > 1) asm volatile("" : "+v"(cr[r]), "+v"(cg_[r]), "+v"(cb[r])::"memory");  // pinned here
            }
        }
    }
}

// NT sub-steps in flight (NT divides CH; R = 1, SPLIT = 1): a ring of NT tap sets, sub-step
// s + NT - 1 issued while sub-step s blends, the issue running into the next chunk (whose
// homography is then held beside the current one).  The kernel is latency-bound with its
// occupancy pinned at 4 waves/SIMD by the LDS slots, so VGPRs up to 128 cost nothing: more
// loads in flight per wave is the lever the A/B ping-pong (NT = 2) leaves unused.
template <int CH, int NT, bool GUARD>
__device__ __forceinline__ void render_chunk_wave_ring(const float* __restrict__ view, const RenderGeom& g,
                                                       const ChunkGeom& cg, const float* __restrict__ hs,
                                                       f32x4* __restrict__ slot, int tx0, int y, int lane, float& cr,
                                                       float& cg_, float& cb, float4* __restrict__ ck,
                                                       int64_t ck_stride) {
    static_assert(CH % NT == 0 && NT >= 2, "the ring position of a sub-step must be static");
    constexpr int PPS = kWave / CH;
    const int j = lane % CH, i = lane / CH;
    const float fy = (float)y;
    const int nchunk = (g.P + CH - 1) / CH;
    float hc[9];  // this chunk's homography (per lane: plane c*CH + j); the next one's is re-read from LDS
    auto load_h = [&](int c, float* d) {
        const int p = min(c * CH + j, g.P - 1);
#pragma unroll
        for (int k = 0; k < 9; ++k) d[k] = hs[p * 9 + k];
    };
    auto issue = [&](int c, int k, const float* hh, ChunkTaps& ts) {
        float px, py;
        chunk_pos<GUARD>(hh, (float)(tx0 + k * PPS + i), fy, g, px, py);
        issue_taps_chunk(make_rsrc(view + (int64_t)c * CH * 4, cg.rec_bytes), g, cg, j, c * CH + j < g.P, px, py, ts);
    };
    auto put = [&](int k, const ChunkTaps& ts) { slot[(k * PPS + i) * (CH + 1) + j] = blend_chunk(ts); };
    auto over_px = [&](const f32x4& s, bool first) {
        const float a = first ? 1.0f : s[3];
        const float om = 1.0f - a;
        cr = over(s[0], a, om, cr);
        cg_ = over(s[1], a, om, cg_);
        cb = over(s[2], a, om, cb);
    };
    ChunkTaps T[NT];
    load_h(0, hc);
#pragma unroll
    for (int k = 0; k + 1 < NT; ++k) issue(0, k, hc, T[k]);
    for (int c = 0; c < nchunk; ++c) {
        const int cn = c + 1 < nchunk ? c + 1 : c;  // past the end: re-issue (cached, unused)
        if (ck && c > 0) ck[c * ck_stride] = make_float4(cr, cg_, cb, 0.0f);
#pragma unroll
        for (int k = 0; k < CH; ++k) {
            const int ka = k + NT - 1;  // the sub-step issued now
            if (ka < CH) {
                issue(c, ka, hc, T[ka % NT]);
            } else {
                float hn[9];
                load_h(cn, hn);
                issue(cn, ka - CH, hn, T[ka % NT]);
            }
            __builtin_amdgcn_sched_barrier(0);
            put(k, T[k % NT]);
            __builtin_amdgcn_sched_barrier(0);
        }
        // composite (lane = pixel): planes c*CH .. c*CH+CH-1, back to front
        const f32x4* row = slot + lane * (CH + 1);
        if (c * CH + CH <= g.P) {
#pragma unroll
            for (int j0 = 0; j0 < CH; j0 += 4) {
                f32x4 sv[4];
#pragma unroll
                for (int jj = 0; jj < 4; ++jj) sv[jj] = row[j0 + jj];
#pragma unroll
                for (int jj = 0; jj < 4; ++jj) over_px(sv[jj], c == 0 && j0 + jj == 0);
            }
        } else {
            for (int jj = 0; c * CH + jj < g.P; ++jj) over_px(row[jj], c * CH + jj == 0);
        }
        load_h(cn, hc);
    }
}

// Vertical strips with tap reuse (round 4, CH = 8): a wave owns an 8 x 8 pixel strip and
// its sub-step k is ROW k of the strip (8 columns x the chunk's 8 planes), so sub-step k+1
// samples each lane's (column, plane) one row below sub-step k.  When a lane's tap origin
// moved exactly one texel row down (the common case at near-unit vertical scale), its
// north taps are the south taps it gathered for row k, already in registers; the north-tap
// gathers are issued only when some lane of the wave needs its own (wave-uniform branch,
// render_rows_kernel's vertical reuse).  Each tap instruction still covers 8 pixels x 8
// consecutive planes (whole 128-B lines where the planes share a texel), so coalescing is
// render_chunk_wave's; the composite reads the same slot rows (slot row = k*8 + column =
// the lane of pixel (column, row k)).  Identical arithmetic: shared taps are the same
// texels' values, so frames and checkpoints are bit-identical to render_chunk_wave's.
struct StripTaps {
    f32x4 a, b, c, d;  // NW, NE (own, when some lane of the wave needs them), SW, SE
    float wx, wy;
    int key;           // clamped tap origin iy * kstride + ix
    bool sh;           // this lane's NW, NE = the previous row's SW, SE
    bool own;          // wave-uniform: some lane gathered its own north taps
};

// issue_taps_chunk for a strip row: the south taps always, the north taps only where some
// lane of the wave does not continue the previous row (t.own).  Returns the number of taps
// inside the image (whether gathered or shared: the backward's pair count).
__device__ __forceinline__ int issue_taps_strip(__amdgpu_buffer_rsrc_t r, const RenderGeom& g, const ChunkGeom& cg,
                                                int jt, bool live, float px, float py, int kstride, int prev_key,
                                                bool can_share, StripTaps& t) {
    const float fx0 = floorf(px), fy0 = floorf(py);
    t.wx = px - fx0;
    t.wy = py - fy0;
    const int ix = (int)__builtin_amdgcn_fmed3f(fx0, -2.0f, (float)g.W);
    const int iy = (int)__builtin_amdgcn_fmed3f(fy0, -2.0f, (float)g.H);
    const bool x0 = (unsigned)ix < (unsigned)g.W, x1 = (unsigned)(ix + 1) < (unsigned)g.W;
    const bool y0 = live && (unsigned)iy < (unsigned)g.H, y1 = live && (unsigned)(iy + 1) < (unsigned)g.H;
    const int off = (int)(((unsigned)__mul24(iy, cg.row_t) + (unsigned)__mul24(ix, cg.pix_t) + (unsigned)jt) * 16u);
    const int pb = cg.pix_t * 16, rb = cg.row_t * 16;
    t.key = iy * kstride + ix;
    t.sh = can_share && t.key == prev_key + kstride;
    t.c = llvm_raw_buffer_load_v4f32(r, (x0 && y1) ? off + rb : kOOB, 0, 0);
    t.d = llvm_raw_buffer_load_v4f32(r, (x1 && y1) ? off + rb + pb : kOOB, 0, 0);
    t.own = __builtin_amdgcn_ballot_w64(!t.sh) != 0;
    if (t.own) {  // wave-uniform: some lane needs its own north taps
        t.a = llvm_raw_buffer_load_v4f32(r, (!t.sh && x0 && y0) ? off : kOOB, 0, 0);
        t.b = llvm_raw_buffer_load_v4f32(r, (!t.sh && x1 && y0) ? off + pb : kOOB, 0, 0);
    }
    return ((int)x0 + (int)x1) * ((int)y0 + (int)y1);
}

// the blended sample of a strip row; pc, pd: the previous row's south taps of this lane
__device__ __forceinline__ f32x4 blend_strip(const StripTaps& t, const f32x4& pc, const f32x4& pd) {
    ChunkTaps u;
    u.a = pc;  // every lane continues (the common case): no per-lane select
    u.b = pd;
    u.c = t.c;
    u.d = t.d;
    u.wx = t.wx;
    u.wy = t.wy;
    if (t.own) {
        asm volatile("");  // keeps this a real (wave-uniform) branch
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            u.a[q] = t.sh ? pc[q] : t.a[q];
            u.b[q] = t.sh ? pd[q] : t.b[q];
        }
    }
    return blend_chunk(u);
}

// SR strip rows (8 or 16: a chunk's sub-steps, one composite phase per 8 rows) and a ring of
// NT rows in flight (row k + NT - 1 issued while row k blends, running on into the next chunk).
template <bool GUARD, int SR, int NT>
__device__ __forceinline__ void render_chunk_wave_strip(const float* __restrict__ view, const RenderGeom& g,
                                                        const ChunkGeom& cg, const float* __restrict__ hs,
                                                        f32x4* __restrict__ slot, int sx0, int sy0, int lane,
                                                        float (&cr)[SR / 8], float (&cg_)[SR / 8], float (&cb)[SR / 8],
                                                        float4* __restrict__ ck, int64_t ck_stride, int64_t ck_half,
                                                        int nhk) {
    constexpr int CH = 8;
    static_assert(SR % 8 == 0 && NT >= 2 && NT <= SR, "strip shape");
    const int j = lane % CH, i = lane / CH;
    const float fx = (float)min(sx0 + i, g.W - 1);  // columns past the frame recompute the last (not stored)
    const int nchunk = (g.P + CH - 1) / CH;
    const int kstride = g.W + 8;  // ix in [-2, W]: the key is injective
    auto load_h = [&](int c, float* d) {
        const int p = min(c * CH + j, g.P - 1);
#pragma unroll
        for (int k = 0; k < 9; ++k) d[k] = hs[p * 9 + k];
    };
    // row k of chunk c: pixel (sx0 + i, sy0 + k), plane c*CH + j (issue_taps_chunk's taps)
    auto issue = [&](int c, int k, const float* hh, int prev_key, bool can_share, StripTaps& t) {
        float px, py;
        chunk_pos<GUARD>(hh, fx, (float)min(sy0 + k, g.H - 1), g, px, py);
        issue_taps_strip(make_rsrc(view + (int64_t)c * CH * 4, cg.rec_bytes), g, cg, j, c * CH + j < g.P, px, py,
                         kstride, prev_key, can_share, t);
    };
    StripTaps T[NT];
    f32x4 sc = {0.f, 0.f, 0.f, 0.f}, sd = sc;  // the previous row's south taps
    float hc[9];
    load_h(0, hc);
#pragma unroll
    for (int k = 0; k + 1 < NT; ++k) issue(0, k, hc, k ? T[k - 1].key : 0, k > 0, T[k]);
    for (int c = 0; c < nchunk; ++c) {
        const int cn = c + 1 < nchunk ? c + 1 : c;  // past the end: re-issue (cached, unused)
        if (ck && c > 0) {
#pragma unroll
            for (int hh = 0; hh < SR / 8; ++hh)
                if (hh < nhk) ck[c * ck_stride + hh * ck_half] = make_float4(cr[hh], cg_[hh], cb[hh], 0.0f);
        }
#pragma unroll
        for (int k = 0; k < SR; ++k) {
            const int ka = k + NT - 1;  // the row issued now
            if (ka < SR) {
                issue(c, ka, hc, T[(ka - 1) % NT].key, true, T[ka % NT]);
            } else {
                float hn[9];
                load_h(cn, hn);  // the next chunk's homography (LDS)
                issue(cn, ka - SR, hn, T[(ka - 1) % NT].key, ka > SR, T[ka % NT]);
            }
            asm volatile("" ::: "memory");  // no later row's loads above this point
            __builtin_amdgcn_sched_barrier(0);
            slot[((k % 8) * CH + i) * (CH + 1) + j] = blend_strip(T[k % NT], sc, sd);
            sc = T[k % NT].c;
            sd = T[k % NT].d;
            asm volatile("" ::: "memory");
            __builtin_amdgcn_sched_barrier(0);
            if (k % 8 == 7) {
                // composite (lane = pixel (column lane % 8, row 8*hh + lane / 8)): planes
                // c*CH .. c*CH+CH-1, back to front
                const int hh = k / 8;
                const f32x4* row = slot + lane * (CH + 1);
                auto over_px = [&](const f32x4& s, bool first) {
                    const float a = first ? 1.0f : s[3];
                    const float om = 1.0f - a;
                    cr[hh] = over(s[0], a, om, cr[hh]);
                    cg_[hh] = over(s[1], a, om, cg_[hh]);
                    cb[hh] = over(s[2], a, om, cb[hh]);
                };
                if (c * CH + CH <= g.P) {
#pragma unroll
                    for (int j0 = 0; j0 < CH; j0 += 4) {
                        f32x4 sv[4];
#pragma unroll
                        for (int jj = 0; jj < 4; ++jj) sv[jj] = row[j0 + jj];
#pragma unroll
                        for (int jj = 0; jj < 4; ++jj) over_px(sv[jj], c == 0 && j0 + jj == 0);
                    }
                } else {
                    for (int jj = 0; c * CH + jj < g.P; ++jj) over_px(row[jj], c * CH + jj == 0);
                }
                if (SR > 8) asm volatile("" : "+v"(cr[hh]), "+v"(cg_[hh]), "+v"(cb[hh])::"memory");  // pinned here
            }
        }
        if constexpr (SR % NT != 0) {  // the next chunk's rows sit at ring positions SR % NT ..: rotate
            StripTaps tmp[NT];
#pragma unroll
            for (int q = 0; q < NT; ++q) tmp[q] = T[(q + SR) % NT];
#pragma unroll
            for (int q = 0; q < NT; ++q) T[q] = tmp[q];
        }
        load_h(cn, hc);
    }
}

constexpr int kStripTX = 32;  // block tile width of the strip kernels (4 strips side by side)

// One block = 4 waves = a 32 x SR output tile of one view (wave w: the 8 x SR strip at column
// 8w); XCD-aware (tile, view) order, tile-level division proof.  Dynamic LDS as
// render_chunk_kernel<8, 1, 1>.
template <int SR, int NT>
__global__ __launch_bounds__(256, 3) void render_chunk_strip_kernel(const float* __restrict__ mpi, int64_t view_stride,
                                                                    RenderGeom g, ChunkGeom cg, int V,
                                                                    const float* __restrict__ homs,
                                                                    float* __restrict__ out,
                                                                    float4* __restrict__ ckpt, int h_lds = 1) {
    extern __shared__ float4 chunk_lds[];
    f32x4* slots = reinterpret_cast<f32x4*>(chunk_lds);
    // the view's homographies in LDS beside the slots, or (h_lds == 0: more planes than fit, the
    // backward's checkpoint pass) read from global memory through the caches
    float* hl = reinterpret_cast<float*>(chunk_lds) + chunk_slot_floats<8, 1>();
    const int tiles_x = (g.W + kStripTX - 1) / kStripTX;
    const int lb = xcd_logical_block(blockIdx.x, gridDim.x);
    const int v = lb % V;
    const int tile = lb / V;
    const int tx0 = (tile % tiles_x) * kStripTX, ty0 = (tile / tiles_x) * SR;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & (kWave - 1);
    const float* hv = homs + (int64_t)v * g.P * 9;
    if (h_lds)
        for (int k = threadIdx.x; k < g.P * 9; k += 256) hl[k] = hv[k];
    const float* hs = h_lds ? hl : hv;
    const float x0 = (float)tx0, x1 = (float)min(tx0 + kStripTX - 1, g.W - 1);
    const float y0 = (float)ty0, y1 = (float)min(ty0 + SR - 1, g.H - 1);
    bool ok = true, dd = true;
    for (int p = (int)threadIdx.x; p < g.P; p += 256) {
        const float* hp = hv + (int64_t)p * 9;
        const bool safe = div2_rect_safe(hp, x0, x1, y0, y1);
        ok = ok && safe;
        dd = dd && safe && tile_dead(hp, x0, x1, y0, y1, g);
    }
    const bool proven = __syncthreads_and(ok);  // also publishes hs
    const bool dead = __syncthreads_and(dd);
    const int sx0 = tx0 + wave * 8;
    if (sx0 >= g.W) return;  // whole wave; no barrier follows
    const float* view = mpi + (int64_t)v * view_stride;
    f32x4* slot = slots + wave * kWave * 9;
    const int x = sx0 + (lane & 7), y = ty0 + (lane >> 3);  // the pixel of half 0 (half h: row y + 8h)
    const int64_t HW = (int64_t)g.H * g.W;
    // checkpoints [V][nchunk][H][W]: half h of this lane at ck + h * 8W, halves past the frame skipped
    const bool in0 = x < g.W && y < g.H;
    float4* ck = (ckpt && in0) ? ckpt + ((int64_t)v * ((g.P + 7) / 8)) * HW + (int64_t)y * g.W + x : nullptr;
    float cr[SR / 8], cgr[SR / 8], cb[SR / 8];
#pragma unroll
    for (int hh = 0; hh < SR / 8; ++hh) cr[hh] = cgr[hh] = cb[hh] = -0.0f;
    const int nhk = min(SR / 8, (g.H - y + 7) / 8);  // halves of this lane inside the frame
    if (dead) {  // every tap of every plane is outside the image (render.hip tile_dead): zero samples
        float r0 = -0.0f, g0 = -0.0f, b0 = -0.0f, t0 = 1.0f;
        for (int c = 0; c * 8 < g.P; ++c) {
            if (ck && c > 0)
                for (int hh = 0; hh < nhk; ++hh) ck[c * HW + hh * 8 * (int64_t)g.W] = make_float4(r0, g0, b0, 0.0f);
            composite_zero<false>(c * 8, min(c * 8 + 8, g.P), c == 0, r0, g0, b0, t0);
        }
#pragma unroll
        for (int hh = 0; hh < SR / 8; ++hh) {
            cr[hh] = r0; cgr[hh] = g0; cb[hh] = b0;
        }
    } else if (proven)
        render_chunk_wave_strip<false, SR, NT>(view, g, cg, hs, slot, sx0, ty0, lane, cr, cgr, cb, ck, HW,
                                               8 * (int64_t)g.W, nhk);
    else
        render_chunk_wave_strip<true, SR, NT>(view, g, cg, hs, slot, sx0, ty0, lane, cr, cgr, cb, ck, HW,
                                              8 * (int64_t)g.W, nhk);
#pragma unroll
    for (int hh = 0; hh < SR / 8; ++hh) {
        if (x < g.W && y + 8 * hh < g.H) {
            float* o = out + (((int64_t)v * g.H + y + 8 * hh) * g.W + x) * 3;
            o[0] = cr[hh];
            o[1] = cgr[hh];
            o[2] = cb[hh];
        }
    }
}

// One block = 4 waves = a 64 x 4R output tile of one view (wave w: rows w*R .. w*R+R-1 of
// the tile); blocks in render_packed_kernel's XCD-aware (tile, view) order.  Dynamic LDS:
// chunk_slot_floats<CH, SPLIT>() + P*9 floats.
template <int CH, int SPLIT, int R, int NT = 2>
__global__ __launch_bounds__(256, SPLIT == 2 ? 6 : 4) void render_chunk_kernel(const float* __restrict__ mpi, int64_t view_stride,
                                                           RenderGeom g, ChunkGeom cg, int V,
                                                           const float* __restrict__ homs,
                                                           float* __restrict__ out,
                                                           float4* __restrict__ ckpt) {
    extern __shared__ float4 chunk_lds[];
    f32x4* slots = reinterpret_cast<f32x4*>(chunk_lds);
    float* hs = reinterpret_cast<float*>(chunk_lds) + chunk_slot_floats<CH, SPLIT>();
    constexpr int TH = kTileY * R;
    const int tiles_x = (g.W + kTileX - 1) / kTileX;
    const int lb = xcd_logical_block(blockIdx.x, gridDim.x);
    const int v = lb % V;
    const int tile = lb / V;
    const int tx0 = (tile % tiles_x) * kTileX, ty0 = (tile / tiles_x) * TH;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & (kWave - 1);
    const float* hv = homs + (int64_t)v * g.P * 9;
    for (int k = threadIdx.x; k < g.P * 9; k += 256) hs[k] = hv[k];
    // block prologue: prove the fast division for the tile, all planes at once
    const float x0 = (float)tx0, x1 = (float)min(tx0 + kTileX - 1, g.W - 1);
    const float y0 = (float)ty0, y1 = (float)min(ty0 + TH - 1, g.H - 1);
    bool ok = true;
    for (int p = (int)threadIdx.x; p < g.P; p += 256) ok = ok && div2_rect_safe(hv + (int64_t)p * 9, x0, x1, y0, y1);
    const bool proven = __syncthreads_and(ok);  // also publishes hs
    const int y = ty0 + wave * R;
    if (y >= g.H) return;  // whole wave; no barrier follows
    const int nrows = min(R, g.H - y);
    const float* view = mpi + (int64_t)v * view_stride;
    f32x4* slot = slots + wave * (kWave / SPLIT) * (CH + 1);
    float cr[R], cgr[R], cb[R];
#pragma unroll
    for (int r = 0; r < R; ++r) cr[r] = cgr[r] = cb[r] = -0.0f;
    const int x = tx0 + lane;
    // checkpoints [V][nchunk][H][W] (nullptr: inference; SPLIT = 1 only: lane = pixel)
    const int64_t HW = (int64_t)g.H * g.W;
    float4* ck = (ckpt && x < g.W) ? ckpt + ((int64_t)v * ((g.P + CH - 1) / CH)) * HW + (int64_t)y * g.W + x : nullptr;
    if constexpr (NT > 2 && R == 1 && SPLIT == 1) {
        if (proven)
            render_chunk_wave_ring<CH, NT, false>(view, g, cg, hs, slot, tx0, y, lane, cr[0], cgr[0], cb[0], ck, HW);
        else
            render_chunk_wave_ring<CH, NT, true>(view, g, cg, hs, slot, tx0, y, lane, cr[0], cgr[0], cb[0], ck, HW);
    } else if (proven) {
        render_chunk_wave<CH, SPLIT, R, false>(view, g, cg, hs, slot, tx0, y, nrows, lane, cr, cgr, cb, ck, HW);
    } else {
        render_chunk_wave<CH, SPLIT, R, true>(view, g, cg, hs, slot, tx0, y, nrows, lane, cr, cgr, cb, ck, HW);
    }
    if (x < g.W) {
#pragma unroll
        for (int r = 0; r < R; ++r) {
            if (r < nrows) {
                float* o = out + (((int64_t)v * g.H + y + r) * g.W + x) * 3;
                o[0] = cr[r];
                o[1] = cgr[r];
                o[2] = cb[r];
            }
        }
    }
}

}  // namespace mpiv
