// render_bwd.hip -- d(render)/d(MPI): the adjoint of the fused warp + over-composite
// (autograd of mpi_render_view_torch, utils.py:267-294, w.r.t. rgba_layers), BIT-EXACT
// to the reference's autograd on CPU (oracle/mpiv_oracle.c oracle_render_backward,
// pinned to tests/golden/grad.npz).
//
// The reference's gradient is a float sum per source texel whose ORDER is fixed by
// ATen's grid_sampler_2d_backward CPU kernel: per (plane, view) slice the output
// pixels are walked in flat chunks of 8; per chunk and channel the corners nw, ne,
// sw, se are scattered over the chunk's lanes in order.  So texel t's sum runs over its
// contributors sorted by the key (pixel/8, corner, pixel%8), from +0.  A scatter with
// float atomics would add in arrival order; here every texel GATHERS its contributors in
// that order instead.  Three steps per view, reading the reference's [B,H,W,P,4] tensor
// in place (no pack):
//
//  1. chain  (bwd_chain_kernel; render_chunk.hip's lane mapping: lanes = (pixel, plane
//            of an 8-plane chunk), so a tap instruction reads whole 128-B pixel lines).
//            Pass 1 composites planes 0..P-1 like the forward and checkpoints the colour
//            before every chunk; pass 2 walks the chunks back to front, re-samples each
//            one, rebuilds its prefixes out_{p-1} from the checkpoint in registers and runs
//            autograd's Mul/Rsub backward over it: d rgb = g*a, d a = sum(g*rgb) +
//            -(sum(g*out_{p-1})), g *= (1 - a).  Only d s_p (16 B per plane-pixel) is
//            written.  It also counts every (sample, in-image tap) pair: the number of
//            (texel, contributor) pairs step 2 must find.
//  2. gather (bwd_gather_kernel): a block owns a 64x4 texel tile of kGPl = 4 planes.  Per plane
//            it maps the tile (one texel margin) back through the inverse homography to a
//            box of output pixels, recomputes their sample positions with the forward's
//            recipe (bit-identical) and stages (nw-tap bucket, fractions, d s) in LDS; each
//            texel then scans the pixels of ITS window (the inverse image of the 2x2 texels
//            whose samples can touch it) in pixel order, collects the hits of one 8-pixel
//            chunk in a 32-bit mask indexed (corner, pixel%8) and adds them in mask-bit
//            order -- exactly the reference's key order.  A texel's kGPl planes leave as one
//            16*kGPl-B run (64 B).  Found pairs are counted.
//  3. check  (bwd_check_kernel): the windows come from float inverse maps, so they are a
//            guess that the count makes exact: every found pair is genuine and found at
//            most once, so found == truth iff nothing was missed.  On a mismatch (or a
//            geometry the gather refuses: plane behind the camera over a tile, boxes beyond
//            LDS, a window whose 8-pixel chunks wrap rows) a device flag turns on the
//            fallback: the general bucket pipeline below (counting sort of every sample by
//            its nw tap, per-bucket pixel order, per-texel merge of the four buckets),
//            launched always but returning at once while the flag is clear, over plane
//            chunks so its workspace stays a fraction of d s.
// Every product and sum is a single fp32 rounding written out explicitly (the library
// builds with -ffp-contract=off).
#include "mpiv_common.hpp"

namespace mpiv {

#ifndef MPIV_BWD_NT
#define MPIV_BWD_NT 0  // A/B: non-temporal stores of the d samples (chain) and of d MPI (gather)
#endif
__device__ __forceinline__ void bwd_store(float4* p, const float4& v) {
    if (MPIV_BWD_NT)
        __builtin_nontemporal_store(f32x4{v.x, v.y, v.z, v.w}, reinterpret_cast<f32x4*>(p));
    else
        *p = v;
}

#ifndef MPIV_BWD_NTOUT
#define MPIV_BWD_NTOUT 0  // A/B: non-temporal stores of the gather's d MPI only
#endif
#ifndef MPIV_GFRAC
#define MPIV_GFRAC 0  // A/B: the gather stages fractions (2 floats) instead of the 4 corner weights
#endif
#ifndef MPIV_GPF2
#define MPIV_GPF2 0  // A/B: the gather loads each pass's d samples during the previous texel phase
#endif
constexpr int kGridVec = 8;        // grid_sampler_2d_backward chunk width (oracle.GRID_VEC)
constexpr int kBwdCH = 8;          // chain: planes per chunk
constexpr int kGTW = 64;           // gather: texel tile width (a wave = one tile row)
#ifndef MPIV_GTH
#define MPIV_GTH 4
#endif
constexpr int kGTH = MPIV_GTH;     // gather: waves per block (a texel row each)
// two texel rows per wave (round 4, profiles/r04_bwd_gather_ab.jsonl): each thread sums two
// independent texels per pass (64 x 8 tiles, 1.4x staged pixels per texel instead of 1.55x),
// 112 VGPRs at 4 waves/SIMD: backward 2.68 vs 2.81 ms, bit-identical
#ifndef MPIV_GTR
#define MPIV_GTR 2
#endif
constexpr int kGTR = MPIV_GTR;     // gather: texel rows per wave (rows w, w + kGTH, ...: a tile of kGTY rows)
constexpr int kGTY = kGTH * kGTR;  // gather: tile rows
constexpr int kGThreads = kGTW * kGTH;
// gather tile constants (overridable for A/B builds, tools/gpu_ab_lib.sh); measured on
// config 4 (profiles/r02_bwd_gather_ab.txt): 4 planes x 736 staged pixels at 6 waves/SIMD
// 2.97 ms per backward, 8 planes x 1024 at 4 waves 3.40, 8 waves (any shape) spills.  Round 3
// (profiles/r03_bwd_gather_ab.txt): the staging's d-sample loads issued ahead of the positions
// need 5 waves/SIMD (at 6 the allocator spills): gather 1.67 vs 1.76 ms
#ifndef MPIV_GPL
#define MPIV_GPL 4
#endif
#ifndef MPIV_GCAP
#define MPIV_GCAP 736
#endif
#ifndef MPIV_GLB
#define MPIV_GLB 4
#endif
#ifndef MPIV_GLBS
#define MPIV_GLBS 3  // bwd_gather_ws_kernel: 512-thread blocks per CU (50 KiB of LDS each)
#endif
#ifndef MPIV_GSI
#define MPIV_GSI 3  // staged pixels per thread whose d samples are loaded ahead of the positions (all of
                    // them: round 4 with two texel rows per wave, 2.51 vs 2.69 ms; r04_bwd_gather_ab.jsonl)
#endif
constexpr int kGPl = MPIV_GPL;     // gather: planes per block (a texel's kGPl planes are one 16*kGPl-B run)
static_assert(kBwdCH % kGPl == 0, "plane groups start at multiples of kBwdCH: a gather block never straddles two");
constexpr int kGCap = MPIV_GCAP;   // gather: output pixels staged per pass
constexpr int kGMaxBox = 64 * kGCap;  // gather: larger boxes (extreme magnification) -> fallback
constexpr int kCtrSlots = 64;      // the two pair counters are spread over 64 words each
constexpr unsigned long long kUnsafe = 1ull << 40;  // > any truth count: forces the fallback

constexpr int kScanItems = 16;     // fallback: items per thread in the bucket scan
constexpr int kScanBlock = 256;
constexpr int kScanTile = kScanItems * kScanBlock;
constexpr int kSmallBucket = 32;   // fallback: larger buckets are sorted by a whole block

struct BwdWs {
    float4* ds;    // [P][HW]  d sample (d rgb, d a) per plane-pixel; in plane groups only the group's
                   //          planes ds_p0 .. ds_p0 + GP - 1 (index through ds_plane)
    int ds_p0 = 0;
    float4* ckpt;  // [nchunk][HW] composited colour before chunk c (c >= 1)
    float* inv;    // [P][12]  texel -> output pixel inverse map (9 floats), [9] = valid
    int4* box;     // [P][tiles] gather pixel box (x0, x1, y0, y1); x0 = -2: the block cannot gather
    unsigned long long* truth;  // [kCtrSlots] (sample, in-image tap) pairs
    unsigned long long* found;  // [kCtrSlots] (texel, contributor) pairs gathered
    int* flag;     // [0] 1: the fallback recomputes every plane of the view; [1], [2] the fallback's
                   // ticket and completion counters; [3] 1: this view's fallback aborted (a wait
                   // outlasted its poll limit); [4] views aborted in this call (bwd_fallback_kernel)
    int* sink = nullptr;    // the device's page-locked abort flag (mpiv_render_backward_abort_flag), set to 1
                            // by an aborted view's NaN fill; nullptr: not mapped
    int* vcount = nullptr;  // where the fallback counts an aborted view (flag + 4; nullptr: the overlapped
                            // schedule counts views in bwd_poison_kernel instead)
    // fallback: bucket pipeline over chunks of pc planes
    int pc;
    int* key;      // [pc][HW] nw-tap bucket in the (H+1) x (W+1) grid, -1 = no tap in the image;
                   //          after the fill: merge-sort scratch (same offsets as ids)
    int* count;    // [pc*K]   bucket sizes; zero after every fill
    int* offs;     // [pc*K+1] exclusive scan of count
    int* ids;      // [pc*HW]  pixel ids grouped by bucket, sorted within a bucket
    int* bsum;     // scan block sums
    int* big;      // [0] = number of large buckets, [1..] their indices
};

// the d samples of plane p (an absolute plane number) in the workspace's window
__device__ __forceinline__ float4* ds_plane(const BwdWs& ws, int p, int64_t HW) {
    return ws.ds + (int64_t)(p - ws.ds_p0) * HW;
}

// ---- 1. chain: forward recompute + over-chain adjoint, in place ----------------------

// sample position with the forward kernels' recipe: MODE 0 = the reference's plain
// divisions (H or W < 2), 1 = fast recipe with the per-sample division guard, 2 = fast
// recipe with the division proven for the whole tile (render.hip div2_rect_safe)
template <int MODE>
__device__ __forceinline__ void bwd_pos(const float* h, float fx, float fy, const RenderGeom& g, float& px,
                                        float& py) {
    if (MODE == 0)
        hom_sample_pos(h, fx, fy, g.hm1, g.wm1, g.half_w, g.half_h, px, py);
    else
        chunk_pos<MODE == 1>(h, fx, fy, g, px, py);
}

// CK: the forward's checkpoints (mpiv_render_train, [nchunk][HW] of this view) replace
// pass 1; every sample is then issued (and its taps counted) in pass 2 only.
// R rows per wave (render_chunk.hip's row grouping): rows y0 .. y0+R-1 of the wave's 64
// columns with the chunk loop outside the row loop (row r+1's north taps come from L1/L2);
// rows past the frame (nrows < R, wave-uniform) re-sample the last row, uncounted and unstored.
template <int MODE, bool CK, int R>
__device__ __forceinline__ void bwd_chain_wave(const float* __restrict__ view, const RenderGeom& g,
                                               const ChunkGeom& cg, const float* __restrict__ hs,
                                               f32x4* __restrict__ slot, int tx0, int y0, int nrows_, int lane,
                                               const float* __restrict__ dout, const float4* __restrict__ ck,
                                               const BwdWs& ws) {
    constexpr int CH = kBwdCH, PPS = kWave / CH;
    const int nrows = R == 1 ? 1 : nrows_;  // wave-uniform
    const int j = lane % CH, i = lane / CH;
    const int n = (g.P + CH - 1) / CH;
    const int64_t HW = (int64_t)g.H * g.W;
    const int x = tx0 + lane;  // this lane's pixel in the composite phases
    const bool xin = x < g.W;
    float h[9];
    auto load_h = [&](int c, float* d) {
        const int p = min(c * CH + j, g.P - 1);
#pragma unroll
        for (int k = 0; k < 9; ++k) d[k] = hs[p * 9 + k];
    };
    auto rsrc = [&](int c) { return make_rsrc(view + (int64_t)c * CH * 4, cg.rec_bytes); };
    int ntap = 0;
    // sub-step k of row r, chunk c: pixel tx0 + k*PPS + i, plane c*CH + j (taps counted once)
    auto issue = [&](int c, int r, int k, const float* hh, ChunkTaps& ts, bool cnt) {
        const int xs = tx0 + k * PPS + i;
        float px, py;
        bwd_pos<MODE>(hh, (float)xs, (float)(y0 + min(r, nrows - 1)), g, px, py);
        const int nt = issue_taps_chunk(rsrc(c), g, cg, j, c * CH + j < g.P, px, py, ts);
        if (cnt && xs < g.W && r < nrows) ntap += nt;
    };
    auto put = [&](int k, const ChunkTaps& ts) { slot[(k * PPS + i) * (CH + 1) + j] = blend_chunk(ts); };
    ChunkTaps A, B;
    // row r of chunk c into the slot; A holds its sub-step 0 on entry and, on exit, sub-step 0
    // of the next row (r + 1 < R) or of row 0 of chunk cn (issued ahead, cn's homography in h)
    auto sample_row = [&](int c, int r, int cn, bool cnt, bool cnt_next) {
#pragma unroll
        for (int k = 0; k < CH; k += 2) {
            issue(c, r, k + 1, h, B, cnt);
            __builtin_amdgcn_sched_barrier(0);
            put(k, A);
            if (k + 2 < CH) {
                issue(c, r, k + 2, h, A, cnt);
            } else if (r + 1 < R) {
                issue(c, r + 1, 0, h, A, cnt);
            } else {
                load_h(cn, h);
                issue(cn, 0, 0, h, A, cnt_next);
            }
            __builtin_amdgcn_sched_barrier(0);
            put(k + 1, B);
        }
    };
    const f32x4* row = slot + lane * (CH + 1);
    // ---- pass 1: planes 0 .. P-1 like the forward (plane 0 replaces the -0 start
    // exactly, render.hip), the colour checkpointed before every chunk.  The last chunk
    // stays in the slot for pass 2 (R == 1); chunk n-2 is issued ahead.
    float cr[R], cgc[R], cb[R];
#pragma unroll
    for (int r = 0; r < R; ++r) cr[r] = cgc[r] = cb[r] = -0.0f;
    if (CK) {
        load_h(n - 1, h);
        issue(n - 1, 0, 0, h, A, true);
    } else {
        load_h(0, h);
        issue(0, 0, 0, h, A, true);
        for (int c = 0; c < n; ++c) {
            const bool last = c == n - 1;
            // R == 1: the last chunk stays in the slot for pass 2, chunk n-2's first sub-step is
            // issued ahead; R > 1: pass 2 re-samples the last chunk (row 0 issued ahead)
#pragma unroll
            for (int r = 0; r < R; ++r) {
                sample_row(c, r, last ? (R == 1 ? max(n - 2, 0) : n - 1) : c + 1, true, !last);
                if (!last && r < nrows) {
#pragma unroll
                    for (int k = 0; k < CH; ++k) {  // a chunk before the last is full
                        const f32x4 s = row[k];
                        const float a = (c == 0 && k == 0) ? 1.0f : s[3];
                        const float om = 1.0f - a;
                        cr[r] = over(s[0], a, om, cr[r]);
                        cgc[r] = over(s[1], a, om, cgc[r]);
                        cb[r] = over(s[2], a, om, cb[r]);
                    }
                    if (xin) ws.ckpt[(int64_t)(c + 1) * HW + (int64_t)(y0 + r) * g.W + x] =
                        make_float4(cr[r], cgc[r], cb[r], 0.0f);
                }
                if (R > 1) asm volatile("" : "+v"(cr[r]), "+v"(cgc[r]), "+v"(cb[r])::"memory");
            }
            if (last) break;
        }
    }
    // ---- pass 2: chunks back to front; over_composite backward (utils.py:149-156 under
    // autograd), planes P-1 .. 0
    float g0[R], g1[R], g2[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
        g0[r] = g1[r] = g2[r] = 0.0f;
        if (xin && r < nrows) {
            const float* d = dout + ((int64_t)(y0 + r) * g.W + x) * 3;
            g0[r] = d[0];
            g1[r] = d[1];
            g2[r] = d[2];
        }
    }
    for (int c = n - 1; c >= 0; --c) {
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const int64_t pix = (int64_t)(y0 + r) * g.W + x;
            float4 pre = make_float4(cr[r], cgc[r], cb[r], 0.0f);  // R == 1, c = n-1: pass 1's colour
            const bool resample = CK || R > 1 || c < n - 1;
            if (resample) {
                if (c == 0)
                    pre = make_float4(-0.0f, -0.0f, -0.0f, 0.0f);
                else if (xin && r < nrows)
                    pre = CK ? ck[(int64_t)c * HW + pix] : ws.ckpt[(int64_t)c * HW + pix];
                // the sample issued ahead for row 0 of chunk c-1 is counted only when every
                // sample is issued here (CK); without checkpoints pass 1 counted it
                sample_row(c, r, c > 0 ? c - 1 : 0, CK, CK && c > 0);
            }
            if (r < nrows) {
                // prefixes out_{p-1} of the chunk's planes, recomputed in the forward's order
                float pr[CH][3];
                pr[0][0] = pre.x;
                pr[0][1] = pre.y;
                pr[0][2] = pre.z;
#pragma unroll
                for (int k = 0; k + 1 < CH; ++k) {
                    const int p = c * CH + k;
                    float rr = pr[k][0], gr = pr[k][1], b = pr[k][2];
                    if (p < g.P) {
                        const f32x4 s = row[k];
                        const float a = p == 0 ? 1.0f : s[3];
                        const float om = 1.0f - a;
                        rr = over(s[0], a, om, rr);
                        gr = over(s[1], a, om, gr);
                        b = over(s[2], a, om, b);
                    }
                    pr[k + 1][0] = rr;
                    pr[k + 1][1] = gr;
                    pr[k + 1][2] = b;
                }
#pragma unroll
                for (int k = CH - 1; k >= 0; --k) {
                    const int p = c * CH + k;
                    if (p < g.P) {
                        const f32x4 s = row[k];
                        float4 d;
                        if (p >= 1) {
                            const float a = s[3], om = 1.0f - a;
                            float s1 = g0[r] * s[0];
                            s1 = s1 + g1[r] * s[1];
                            s1 = s1 + g2[r] * s[2];
                            float s2 = g0[r] * pr[k][0];
                            s2 = s2 + g1[r] * pr[k][1];
                            s2 = s2 + g2[r] * pr[k][2];
                            d = make_float4(g0[r] * a, g1[r] * a, g2[r] * a, s1 + (-s2));
                            g0[r] = g0[r] * om;
                            g1[r] = g1[r] * om;
                            g2[r] = g2[r] * om;
                        } else {
                            d = make_float4(g0[r], g1[r], g2[r], 0.0f);  // plane 0: output = rgb_0, alpha unused
                        }
                        if (xin) bwd_store(ds_plane(ws, p, HW) + pix, d);
                    }
                }
            }
            if (R > 1) asm volatile("" : "+v"(g0[r]), "+v"(g1[r]), "+v"(g2[r])::"memory");
        }
    }
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) ntap += __shfl_xor(ntap, off);
    if (lane == 0 && ntap) atomicAdd(&ws.truth[blockIdx.x % kCtrSlots], (unsigned long long)ntap);
}

// One block = 4 waves = a 64 x 4R output tile of one view (wave w: rows w*R .. w*R+R-1).
// Dynamic LDS: 4 per-wave sample slots (64 x (CH+1) float4) + the view's P homographies.
// MODE 0: generic recipe (H or W < 2); 1: fast recipe, the tile's division proof picks the
// unguarded path.
template <int MODE, bool CK, int R>
__global__ __launch_bounds__(256, R == 1 ? 1 : 4) void bwd_chain_kernel(const float* __restrict__ view, RenderGeom g, ChunkGeom cg,
                                                           const float* __restrict__ homs,
                                                           const float* __restrict__ dout,
                                                           const float4* __restrict__ ck, BwdWs ws, int h_lds) {
    extern __shared__ float4 bwd_lds[];
    f32x4* slots = reinterpret_cast<f32x4*>(bwd_lds);
    // the view's homographies: staged in LDS, or (h_lds == 0: more planes than the LDS holds
    // beside the slots) read from global memory through the caches
    float* hl = reinterpret_cast<float*>(bwd_lds) + 4 * kWave * (kBwdCH + 1) * 4;
    const float* hs = h_lds ? hl : homs;
    constexpr int TH = kTileY * R;
    const int tiles_x = (g.W + kTileX - 1) / kTileX;
    const int tile = xcd_logical_block(blockIdx.x, gridDim.x);
    const int tx0 = (tile % tiles_x) * kTileX, ty0 = (tile / tiles_x) * TH;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & (kWave - 1);
    if (h_lds)
        for (int k = threadIdx.x; k < g.P * 9; k += 256) hl[k] = homs[k];
    bool ok = MODE != 0;
    if (MODE != 0) {
        const float x0 = (float)tx0, x1 = (float)min(tx0 + kTileX - 1, g.W - 1);
        const float y0 = (float)ty0, y1 = (float)min(ty0 + TH - 1, g.H - 1);
        for (int p = (int)threadIdx.x; p < g.P; p += 256) ok = ok && div2_rect_safe(homs + (int64_t)p * 9, x0, x1, y0, y1);
    }
    const bool proven = __syncthreads_and(ok);  // also publishes hs
    const int y = ty0 + wave * R;
    if (y >= g.H) return;  // whole wave; no barrier follows
    const int nrows = min(R, g.H - y);
    f32x4* slot = slots + wave * kWave * (kBwdCH + 1);
    if (MODE == 0)
        bwd_chain_wave<0, CK, R>(view, g, cg, hs, slot, tx0, y, nrows, lane, dout, ck, ws);
    else if (proven)
        bwd_chain_wave<2, CK, R>(view, g, cg, hs, slot, tx0, y, nrows, lane, dout, ck, ws);
    else
        bwd_chain_wave<1, CK, R>(view, g, cg, hs, slot, tx0, y, nrows, lane, dout, ck, ws);
}

// The chain fed the forward's checkpoints, as 8 x 8 strips with vertical tap reuse
// (render_chunk.hip render_chunk_wave_strip, round 4): row k of the strip is sub-step k of a
// chunk, so a lane's north taps are usually the south taps it gathered one row above; the
// composite phases run with lane = pixel (column lane % 8, row lane / 8).  Same samples,
// same adjoint arithmetic, same pair count (every in-image tap of every sample, gathered or
// shared): the d samples are bit-identical to bwd_chain_wave<MODE, true, 1>'s.
// Chunks [c_lo, c_hi) only (a plane group, mpiv_render_backward: groups back to front so the
// d samples of one group at a time fit the workspace): g starts from dout for the top group
// (c_hi == n) and from gbuf otherwise, and leaves in gbuf for the group below (c_lo > 0).
template <int MODE, int SR>
__device__ __forceinline__ void bwd_chain_wave_strip(const float* __restrict__ view, const RenderGeom& g,
                                                     const ChunkGeom& cg, const float* __restrict__ hs,
                                                     f32x4* __restrict__ slot, int sx0, int sy0, int lane,
                                                     const float* __restrict__ dout, const float4* __restrict__ ck,
                                                     const BwdWs& ws, int c_lo, int c_hi, float4* __restrict__ gbuf) {
    constexpr int CH = kBwdCH, NH = SR / 8;
    static_assert(SR % 8 == 0, "strip rows");
    const int j = lane % CH, i = lane / CH;
    const int n = (g.P + CH - 1) / CH;
    const int64_t HW = (int64_t)g.H * g.W;
    const int x = sx0 + (lane & 7), y = sy0 + (lane >> 3);  // this lane's pixel of half 0 (half h: row y + 8h)
    const int64_t pix = (int64_t)y * g.W + x;
    const int64_t hstep = 8 * (int64_t)g.W;
    const bool col_in = sx0 + i < g.W;
    const float fx = (float)min(sx0 + i, g.W - 1);  // columns past the frame recompute the last (uncounted)
    const int kstride = g.W + 8;
    float h[9];
    auto load_h = [&](int c, float* d) {
        const int p = min(c * CH + j, g.P - 1);
#pragma unroll
        for (int k = 0; k < 9; ++k) d[k] = hs[p * 9 + k];
    };
    int ntap = 0;
    // row k of chunk c: pixel (sx0 + i, sy0 + k), plane c*CH + j (taps counted once)
    auto issue = [&](int c, int k, const float* hh, int prev_key, bool can_share, StripTaps& t, bool cnt) {
        const int ys = sy0 + k;
        float px, py;
        bwd_pos<MODE>(hh, fx, (float)min(ys, g.H - 1), g, px, py);
        const int nt = issue_taps_strip(make_rsrc(view + (int64_t)c * CH * 4, cg.rec_bytes), g, cg, j, c * CH + j < g.P,
                                        px, py, kstride, prev_key, can_share, t);
        if (cnt && col_in && ys < g.H) ntap += nt;
    };
    StripTaps A, B;
    f32x4 sc = {0.f, 0.f, 0.f, 0.f}, sd = sc;
    // rows 8*hh .. 8*hh+7 of chunk c into the slot; A holds row 8*hh on entry and, on exit, the
    // next row: 8*hh + 8 of chunk c, or row 0 of chunk cn
    auto sample_half = [&](int c, int hh, int cn, bool cnt_next) {
#pragma unroll
        for (int k = 0; k < 8; k += 2) {
            const int r = 8 * hh + k;
            issue(c, r + 1, h, A.key, true, B, true);
            asm volatile("" ::: "memory");
            __builtin_amdgcn_sched_barrier(0);
            slot[(k * CH + i) * (CH + 1) + j] = blend_strip(A, sc, sd);
            sc = A.c;
            sd = A.d;
            if (k + 2 < 8) {
                issue(c, r + 2, h, B.key, true, A, true);
            } else if (hh + 1 < NH) {
                issue(c, r + 2, h, B.key, true, A, true);
            } else {
                load_h(cn, h);
                issue(cn, 0, h, 0, false, A, cnt_next);
            }
            asm volatile("" ::: "memory");
            __builtin_amdgcn_sched_barrier(0);
            slot[((k + 1) * CH + i) * (CH + 1) + j] = blend_strip(B, sc, sd);
            sc = B.c;
            sd = B.d;
        }
    };
    const f32x4* row = slot + lane * (CH + 1);
    float g0[NH], g1[NH], g2[NH];
    bool in[NH];
#pragma unroll
    for (int hh = 0; hh < NH; ++hh) {
        in[hh] = x < g.W && y + 8 * hh < g.H;
        g0[hh] = g1[hh] = g2[hh] = 0.0f;
        if (in[hh] && c_hi == n) {
            const float* d = dout + (pix + hh * hstep) * 3;
            g0[hh] = d[0];
            g1[hh] = d[1];
            g2[hh] = d[2];
        } else if (in[hh]) {  // the group above left g here
            const float4 gv = gbuf[pix + hh * hstep];
            g0[hh] = gv.x;
            g1[hh] = gv.y;
            g2[hh] = gv.z;
        }
    }
    load_h(c_hi - 1, h);
    issue(c_hi - 1, 0, h, 0, false, A, true);
    // over_composite backward (utils.py:149-156 under autograd), chunks back to front
    for (int c = c_hi - 1; c >= c_lo; --c) {
#pragma unroll
        for (int hh = 0; hh < NH; ++hh) {
            float4 pre = make_float4(-0.0f, -0.0f, -0.0f, 0.0f);
            if (c > 0 && in[hh]) pre = ck[(int64_t)c * HW + pix + hh * hstep];
            // the row issued ahead for chunk c-1 belongs to this group (counted) only above c_lo
            sample_half(c, hh, c > c_lo ? c - 1 : c_lo, c > c_lo);
            float pr[CH][3];  // prefixes out_{p-1} of the chunk's planes, in the forward's order
            pr[0][0] = pre.x;
            pr[0][1] = pre.y;
            pr[0][2] = pre.z;
#pragma unroll
            for (int k = 0; k + 1 < CH; ++k) {
                const int p = c * CH + k;
                float rr = pr[k][0], gr = pr[k][1], b = pr[k][2];
                if (p < g.P) {
                    const f32x4 s = row[k];
                    const float a = p == 0 ? 1.0f : s[3];
                    const float om = 1.0f - a;
                    rr = over(s[0], a, om, rr);
                    gr = over(s[1], a, om, gr);
                    b = over(s[2], a, om, b);
                }
                pr[k + 1][0] = rr;
                pr[k + 1][1] = gr;
                pr[k + 1][2] = b;
            }
#pragma unroll
            for (int k = CH - 1; k >= 0; --k) {
                const int p = c * CH + k;
                if (p < g.P) {
                    const f32x4 s = row[k];
                    float4 d;
                    if (p >= 1) {
                        const float a = s[3], om = 1.0f - a;
                        float s1 = g0[hh] * s[0];
                        s1 = s1 + g1[hh] * s[1];
                        s1 = s1 + g2[hh] * s[2];
                        float s2 = g0[hh] * pr[k][0];
                        s2 = s2 + g1[hh] * pr[k][1];
                        s2 = s2 + g2[hh] * pr[k][2];
                        d = make_float4(g0[hh] * a, g1[hh] * a, g2[hh] * a, s1 + (-s2));
                        g0[hh] = g0[hh] * om;
                        g1[hh] = g1[hh] * om;
                        g2[hh] = g2[hh] * om;
                    } else {
                        d = make_float4(g0[hh], g1[hh], g2[hh], 0.0f);  // plane 0: output = rgb_0, alpha unused
                    }
                    if (in[hh]) bwd_store(ds_plane(ws, p, HW) + pix + hh * hstep, d);
                }
            }
            if (NH > 1) asm volatile("" : "+v"(g0[hh]), "+v"(g1[hh]), "+v"(g2[hh])::"memory");  // pinned here
        }
    }
    if (c_lo > 0) {
#pragma unroll
        for (int hh = 0; hh < NH; ++hh)
            if (in[hh]) gbuf[pix + hh * hstep] = make_float4(g0[hh], g1[hh], g2[hh], 0.0f);
    }
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) ntap += __shfl_xor(ntap, off);
    if (lane == 0 && ntap) atomicAdd(&ws.truth[blockIdx.x % kCtrSlots], (unsigned long long)ntap);
}

// One block = 4 waves = a 32 x SR output tile (wave w: the 8 x SR strip at column 8w); LDS and
// h_lds as bwd_chain_kernel.  Fast recipe only (MODE 1 / 2 by the tile's division proof).
template <int SR>
__global__ __launch_bounds__(256, 1) void bwd_chain_strip_kernel(const float* __restrict__ view, RenderGeom g,
                                                                 ChunkGeom cg, const float* __restrict__ homs,
                                                                 const float* __restrict__ dout,
                                                                 const float4* __restrict__ ck, BwdWs ws, int h_lds,
                                                                 int c_lo, int c_hi, float4* __restrict__ gbuf) {
    extern __shared__ float4 bwd_lds[];
    f32x4* slots = reinterpret_cast<f32x4*>(bwd_lds);
    float* hl = reinterpret_cast<float*>(bwd_lds) + 4 * kWave * (kBwdCH + 1) * 4;
    const float* hs = h_lds ? hl : homs;
    const int tiles_x = (g.W + kStripTX - 1) / kStripTX;
    const int tile = xcd_logical_block(blockIdx.x, gridDim.x);
    const int tx0 = (tile % tiles_x) * kStripTX, ty0 = (tile / tiles_x) * SR;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & (kWave - 1);
    if (h_lds)
        for (int k = threadIdx.x; k < g.P * 9; k += 256) hl[k] = homs[k];
    bool ok = true, dd = true;
    {
        const float x0 = (float)tx0, x1 = (float)min(tx0 + kStripTX - 1, g.W - 1);
        const float y0 = (float)ty0, y1 = (float)min(ty0 + SR - 1, g.H - 1);
        const int p_end = min(g.P, c_hi * kBwdCH);  // the group's planes (the rows issued past it are unused)
        for (int p = c_lo * kBwdCH + (int)threadIdx.x; p < p_end; p += 256) {
            const float* hp = homs + (int64_t)p * 9;
            const bool safe = div2_rect_safe(hp, x0, x1, y0, y1);
            ok = ok && safe;
            dd = dd && safe && tile_dead(hp, x0, x1, y0, y1, g);
        }
    }
    const bool proven = __syncthreads_and(ok);  // also publishes hs
    const bool dead = __syncthreads_and(dd);
    const int sx0 = tx0 + wave * 8;
    if (sx0 >= g.W) return;  // whole wave; no barrier follows
    if (dead) {
        // Round 6: no sample of the tile has an in-image tap in the group's planes (render.hip
        // tile_dead).  Its d samples are never read -- the gather and the fallback sum the contributors
        // of real texels only -- its pair count is 0, and g crosses every plane unchanged (sample +0:
        // a = +0, g * 1 = g); only the hand-over to the group below remains, and where g came from
        // gbuf (c_hi < n) it is already there.
        const int n = (g.P + kBwdCH - 1) / kBwdCH;
        if (c_lo > 0 && c_hi == n) {
            const int x = sx0 + (lane & 7), y = ty0 + (lane >> 3);
#pragma unroll
            for (int hh = 0; hh < SR / 8; ++hh) {
                if (x < g.W && y + 8 * hh < g.H) {
                    const int64_t q = (int64_t)(y + 8 * hh) * g.W + x;
                    gbuf[q] = make_float4(dout[q * 3 + 0], dout[q * 3 + 1], dout[q * 3 + 2], 0.0f);
                }
            }
        }
        return;
    }
    f32x4* slot = slots + wave * kWave * (kBwdCH + 1);
    if (proven)
        bwd_chain_wave_strip<2, SR>(view, g, cg, hs, slot, sx0, ty0, lane, dout, ck, ws, c_lo, c_hi, gbuf);
    else
        bwd_chain_wave_strip<1, SR>(view, g, cg, hs, slot, sx0, ty0, lane, dout, ck, ws, c_lo, c_hi, gbuf);
}

// ---- 2. gather: per-texel sums in the reference's order ------------------------------

// Per plane, the inverse of F = T S H, the map from an output pixel (x, y, 1) to its
// sample position: px = (W/(H-1)) * u/w - 0.5, py = (H/(W-1)) * v/w - 0.5 (the swapped
// normalisation of utils.py:188 and grid_sample's unnormalise, in exact arithmetic).
// F^-1 (x', y', z') of a texel point is (x, y, 1) / w, so z' > 0 exactly where the point is
// the image of pixels in front of the camera.  Computed in double, stored as floats: the
// windows built from it are guesses checked by the pair count.
__device__ __forceinline__ void bwd_plane_inverse(const float* __restrict__ h, double sx, double sy, float* o) {
    double f[9];
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        f[c] = sx * (double)h[c] - 0.5 * (double)h[6 + c];
        f[3 + c] = sy * (double)h[3 + c] - 0.5 * (double)h[6 + c];
        f[6 + c] = (double)h[6 + c];
    }
    double a[9];
    a[0] = f[4] * f[8] - f[5] * f[7];
    a[1] = f[2] * f[7] - f[1] * f[8];
    a[2] = f[1] * f[5] - f[2] * f[4];
    a[3] = f[5] * f[6] - f[3] * f[8];
    a[4] = f[0] * f[8] - f[2] * f[6];
    a[5] = f[2] * f[3] - f[0] * f[5];
    a[6] = f[3] * f[7] - f[4] * f[6];
    a[7] = f[1] * f[6] - f[0] * f[7];
    a[8] = f[0] * f[4] - f[1] * f[3];
    const double det = f[0] * a[0] + f[1] * a[3] + f[2] * a[6];
    bool ok = det != 0.0 && __builtin_isfinite(det);
#pragma unroll
    for (int k = 0; k < 9; ++k) {
        const float v = ok ? (float)(a[k] / det) : 0.0f;
        ok = ok && __builtin_isfinite(v);
        o[k] = v;
    }
    o[9] = ok ? 1.0f : 0.0f;
}

__global__ __launch_bounds__(64) void bwd_inverse_kernel(const float* __restrict__ homs, int P, double sx,
                                                         double sy, float* __restrict__ inv) {
    const int p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= P) return;
    bwd_plane_inverse(homs + (int64_t)p * 9, sx, sy, inv + (int64_t)p * 12);
}

// texel point (X, Y) -> output pixel point; false unless in front of the camera
__device__ __forceinline__ bool inv_map(const float* m, float X, float Y, float& x, float& y) {
    const float z = __builtin_fmaf(m[7], Y, m[6] * X) + m[8];
    const float r = __builtin_amdgcn_rcpf(z);
    x = (__builtin_fmaf(m[1], Y, m[0] * X) + m[2]) * r;
    y = (__builtin_fmaf(m[4], Y, m[3] * X) + m[5]) * r;
    return z > 0.0f && __builtin_isfinite(x) && __builtin_isfinite(y);
}

// Integer pixel range [lo, hi] covering [a - e, b + e], clamped to [cl, ch] (empty: lo > hi).
__device__ __forceinline__ void pix_range(float a, float b, float e, int cl, int ch, int& lo, int& hi) {
    lo = (int)ceilf(__builtin_fmaxf(a - e, (float)cl));
    hi = (int)floorf(__builtin_fminf(b + e, (float)ch));
}

// Per (plane, gather tile): the box of output pixels whose samples can have a nw tap in
// the tile's bucket region [tx0-1, tx0+kGTW] x [ty0-1, ty0+kGTH] (inverse image of its
// corners, widened by `margin`), clamped to the frame; x0 = -2 when the block cannot gather
// the plane (no inverse, a corner behind the camera, a box beyond the staging limits, or an
// 8-pixel chunk wrapping rows across two passes): the check then sends the view to the
// fallback.  x0 > x1 or y0 > y1: no pixel samples the tile.
constexpr int kGTHc = kGTY;
constexpr int kBoxProven = 1 << 30;
// INV (round 6): the plane's inverse computed here (bwd_plane_inverse, the same double arithmetic,
// so the same floats) instead of read from bwd_inverse_kernel's output -- one launch fewer per
// view; the first tile's thread of each plane stores it for the gather.
// zero (round 6, the single-group schedule, which launches this kernel before the chain): block 0
// also zeroes the pair counters and the flag words -- the hipMemsetAsync of the workspace's head
// (1: per view; 2: the call's first view, with the aborted-view count).
template <bool INV = false>
__global__ __launch_bounds__(256) void bwd_box_kernel(RenderGeom g, const float* __restrict__ homs,
                                                      float* __restrict__ inv, int ntiles, int tiles_x,
                                                      float margin, int4* __restrict__ box, double sx = 0.0,
                                                      double sy = 0.0, BwdWs zero_ws = BwdWs{}, int zero = 0) {
    if (zero && blockIdx.x == 0 && threadIdx.x < kCtrSlots) {
        zero_ws.truth[threadIdx.x] = 0;
        zero_ws.found[threadIdx.x] = 0;
        if (threadIdx.x < 16 && (threadIdx.x != 4 || zero == 2)) zero_ws.flag[threadIdx.x] = 0;
    }
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= (int64_t)g.P * ntiles) return;
    const int p = (int)(i / ntiles), tile = (int)(i - (int64_t)p * ntiles);
    const int tx0 = (tile % tiles_x) * kGTW, ty0 = (tile / tiles_x) * kGTHc;
    float iv[10];
    if (INV) {
        bwd_plane_inverse(homs + (int64_t)p * 9, sx, sy, iv);
        if (tile == 0) {
#pragma unroll
            for (int k = 0; k < 10; ++k) inv[(int64_t)p * 12 + k] = iv[k];
        }
    } else {
#pragma unroll
        for (int k = 0; k < 10; ++k) iv[k] = inv[(int64_t)p * 12 + k];
    }
    float m[9];
#pragma unroll
    for (int k = 0; k < 9; ++k) m[k] = iv[k];
    bool bad = iv[9] == 0.0f;
    float xmn = __builtin_inff(), xmx = -__builtin_inff(), ymn = __builtin_inff(), ymx = -__builtin_inff();
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        float xx, yy;
        const bool okc =
            inv_map(m, (float)((c & 1) ? tx0 + kGTW : tx0 - 1), (float)((c & 2) ? ty0 + kGTHc : ty0 - 1), xx, yy);
        bad = bad || !okc;
        xmn = __builtin_fminf(xmn, xx);
        xmx = __builtin_fmaxf(xmx, xx);
        ymn = __builtin_fminf(ymn, yy);
        ymx = __builtin_fmaxf(ymx, yy);
    }
    int bx0 = 0, bx1 = -1, by0 = 0, by1 = -1;
    if (!bad) {
        pix_range(xmn, xmx, margin, 0, g.W - 1, bx0, bx1);
        pix_range(ymn, ymx, margin, 0, g.H - 1, by0, by1);
        const int bw = bx1 - bx0 + 1, bh = by1 - by0 + 1;
        if (bw > 0 && bh > 0) {
            const int rpp = bw <= kGCap ? kGCap / bw : 1;
            bad = bw > kGCap || (int64_t)bw * bh > kGMaxBox ||
                  (bh > rpp && (g.W & 7) && bx0 <= 6 && bx1 >= g.W - 7);
        }
    }
    // bit 30 of y1: the fast division is proven for every pixel of the box (render.hip
    // div2_rect_safe), so the gather's fill needs no per-sample guard
    const bool proven = !bad && bx0 <= bx1 && by0 <= by1 &&
                        div2_rect_safe(homs + (int64_t)p * 9, (float)bx0, (float)bx1, (float)by0, (float)by1);
    box[i] = bad ? make_int4(-2, -3, 0, -1) : make_int4(bx0, bx1, by0, by1 | (proven ? kBoxProven : 0));
}

__device__ __forceinline__ void sort4(unsigned& a, unsigned& b, unsigned& c, unsigned& d) {
    auto cx = [](unsigned& x, unsigned& y) {
        const unsigned lo = min(x, y), hi = max(x, y);
        x = lo;
        y = hi;
    };
    cx(a, b); cx(c, d); cx(a, c); cx(b, d); cx(b, c);
}

// 8-input sorting network (19 comparators; checked exhaustively by the 0-1 principle)
__device__ __forceinline__ void sort8(unsigned* k) {
    auto cx = [&](int a, int b) {
        const unsigned lo = min(k[a], k[b]), hi = max(k[a], k[b]);
        k[a] = lo;
        k[b] = hi;
    };
    cx(0, 1); cx(2, 3); cx(4, 5); cx(6, 7);
    cx(0, 2); cx(1, 3); cx(4, 6); cx(5, 7);
    cx(1, 2); cx(5, 6); cx(0, 4); cx(3, 7);
    cx(1, 5); cx(2, 6);
    cx(1, 4); cx(3, 6);
    cx(2, 4); cx(3, 5);
    cx(3, 4);
}

constexpr int kGTB = kGTW + 1;              // bucket row pitch: nw taps x in [tx0-1, tx0+kGTW-1]
constexpr int kGNB = kGTB * (kGTY + 1);     // nw-tap buckets of a tile
constexpr int kGBCap = 2;                   // entries per bucket list (more: the window scan)
constexpr int kGSI = (kGCap + kGThreads - 1) / kGThreads;  // staged pixels per staging thread
// staged bilinear weights, corner-major: s_w[c * kGWP + q] is corner c's weight of staged pixel q
// (c = nw, ne, sw, se; q = kGCap: the zero slot).  The texel pass reads one corner per key, and
// neighbouring texels read neighbouring staged pixels: consecutive dwords, conflict-free, where
// a pixel-major float4 array puts a 32-lane read on 8 banks (4-way conflicts).
constexpr int kGWP = kGCap + 1;

// One staging pass of plane p over box rows [ra, rb) x columns [bx0, bx0 + bw) by the kGThreads
// threads t of a block (or of its staging waves): each box pixel's sample position with the
// forward's recipe (bit-identical), its nw-tap bucket in the tile's (kGTW+1) x (kGTH+1) grid,
// fractions and d sample into the staged arrays, and its order key pushed onto its bucket's
// list (two entries per bucket, ~0 = free, claimed by LDS compare-and-swap; a third sets
// *ovf).  The pass's d samples are loaded first (MPIV_GSI per thread in flight while the
// positions are computed: issued after each pixel's position, inside the in-tile test, their
// latency was exposed -- 0.32 of the kernel's 1.77 ms, r03).  s_ent must be all ~0 on entry.
// DS = false (bwd_gather_dma_kernel): the d samples arrive in LDS by DMA instead, and only the
// fractions (wx, wy) are staged (s_w[q], s_w[kGWP + q]); the texel pass forms the corner weight.
// PRE (MPIV_GPF2 gather): the d samples were loaded by the caller (pre[i]: staged pixel
// t + i * kGThreads, a pass ahead) instead of here.
template <bool DS = true, bool PRE = false, bool FR = false>
__device__ __forceinline__ void gather_stage_pass(const RenderGeom& g, const BwdWs& ws, const float* __restrict__ hp,
                                                  int p, bool proven, int t, int tx0, int ty0, int bx0, int bw,
                                                  int ra, int rb, int* s_code, float* s_w, float4* s_ds,
                                                  unsigned* s_ent, int* ovf, const f32x4* pre = nullptr) {
    constexpr int TB = kGTB;
    const int64_t HW = (int64_t)g.H * g.W;
    const int np = (rb - ra) * bw;
    const int gbase = (ra * g.W) >> 3;  // the pass's first 8-pixel chunk
    // order keys hold (chunk - gbase) in 16 bits
    if (t == 0 && (int64_t)(rb - ra + 1) * g.W >= ((int64_t)1 << 19)) *ovf = 1;
    const float rbw = 1.0f / (float)bw;
    const __amdgpu_buffer_rsrc_t rds = make_rsrc(ds_plane(ws, p, HW), (int)(HW * 16));
    f32x4 dsv[kGSI];
    if (DS && PRE) {
#pragma unroll
        for (int i = 0; i < kGSI; ++i) dsv[i] = pre[i];
    } else if (DS) {
#pragma unroll
        for (int i = 0; i < (kGSI < MPIV_GSI ? kGSI : MPIV_GSI); ++i) {
            const int q = t + i * kGThreads;
            const int r = (int)(((float)q + 0.5f) * rbw);  // q / bw: q, bw <= 1024, error << 0.5/bw
            const int off = q < np ? ((ra + r) * g.W + bx0 + (q - r * bw)) * 16 : kOOB;
            dsv[i] = llvm_raw_buffer_load_v4f32(rds, off, 0, 0);
        }
    }
    bool ovl = false;
#pragma unroll
    for (int i = 0; i < kGSI; ++i) {
        const int q = t + i * kGThreads;
        const bool qv = q < np;  // no divergent loop exit: pixels past the pass are masked below
        const int r = (int)(((float)q + 0.5f) * rbw);
        const int yy = ra + r, xx = bx0 + (q - r * bw);
        float px, py;
        if (proven)
            render_pos_fast<false>(hp, (float)xx, (float)yy, g, px, py);
        else
            render_pos<true>(hp, (float)xx, (float)yy, g, px, py);
        const float fx0 = floorf(px), fy0 = floorf(py);
        const float lx = fx0 - (float)(tx0 - 1), ly = fy0 - (float)(ty0 - 1);
        const bool in = qv && lx >= 0.0f && lx <= (float)kGTW && ly >= 0.0f && ly <= (float)kGTY;
        const int code = in ? (int)ly * TB + (int)lx : -1;
        if (qv) s_code[q] = code;
        if (in) {
            // the four bilinear weights (issue_taps_padded's products, corner order nw, ne, sw, se):
            // the texel pass reads the one of its corner instead of re-deriving it from fractions
            const float wx = px - fx0, ex = 1.0f - wx;
            const float wy = py - fy0, sy = 1.0f - wy;
            if (DS) {
                if (FR) {  // fractions only (MPIV_GFRAC): the texel pass forms the corner weight
                    s_w[q] = wx;
                    s_w[kGWP + q] = wy;
                } else {
                    s_w[q] = sy * ex;
                    s_w[kGWP + q] = sy * wx;
                    s_w[2 * kGWP + q] = wy * ex;
                    s_w[3 * kGWP + q] = wy * wx;
                }
                if (!PRE && i >= MPIV_GSI)  // past the preloaded pixels (boxes over MPIV_GSI * kGThreads pixels)
                    dsv[i] = llvm_raw_buffer_load_v4f32(rds, (yy * g.W + xx) * 16, 0, 0);
                s_ds[q] = make_float4(dsv[i][0], dsv[i][1], dsv[i][2], dsv[i][3]);
            } else {
                s_w[q] = wx;
                s_w[kGWP + q] = wy;
            }
            const int pix = yy * g.W + xx;
            // order key (never ~0: bits 14-15 are clear) into the first free slot of the bucket
            // (~0 = free; any order: the texel pass sorts)
            const unsigned e = ((unsigned)((pix >> 3) - gbase) << 16) | ((unsigned)(pix & 7) << 11) | (unsigned)q;
            unsigned* ent = s_ent + 2 * code;
            if (atomicCAS(ent, ~0u, e) != ~0u && atomicCAS(ent + 1, ~0u, e) != ~0u) ovl = true;
        }
    }
    if (ovl) *ovf = 1;
}

// One texel-phase pass: texel (tx, ty)'s sum over the pass's contributors, added in the
// reference's key order into a.  The texel is the nw / ne / sw / se tap of the samples in
// buckets bt, bt-1, bt-row, bt-row-1: their <= 8 keys (pixel/8 relative to the pass, corner,
// pixel%8, staged index in the low bits) go through a 4- or 8-input sorting network and are
// added in order.  After a list overflow (magnification) the texel scans its window of the
// inverse map instead, one 8-pixel chunk at a time.
// corner c's bilinear weight of staged pixel q: staged products (s_w corner-major), or (FRAC)
// formed from the staged fractions with issue_taps_padded's products (the same bits)
template <bool FRAC>
__device__ __forceinline__ float staged_weight(const float* s_w, int c, int q) {
    if (!FRAC) return s_w[c * kGWP + q];
    const float wx = s_w[q], wy = s_w[kGWP + q];
    return ((c & 2) ? wy : 1.0f - wy) * ((c & 1) ? wx : 1.0f - wx);
}

template <bool FRAC = false>
__device__ __forceinline__ void gather_texel_pass(const RenderGeom& g, const BwdWs& ws, int p, float margin, int tx,
                                                  int ty, int bt, bool tin, bool ovf, const unsigned* s_ent,
                                                  const int* s_code, const float* s_w, const float4* s_ds, int bx0,
                                                  int bx1, int by0, int by1, int ra, int rb, f32x4& acc,
                                                  unsigned& hits, bool& unsafe) {
    constexpr int TB = kGTB;
    const int bw = bx1 - bx0 + 1;
    if (tin && !ovf) {
        // the texel's <= 8 contributors: buckets t (nw), t-1 (ne), t-row (sw), t-row-1 (se)
        unsigned key[8];  // a free slot (~0) stays ~0 after the corner is or-ed in
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            const int b = bt - (c & 1) - (c >> 1) * TB;
            const uint2 e = reinterpret_cast<const uint2*>(s_ent)[b];
            key[2 * c] = e.x | ((unsigned)c << 14);
            key[2 * c + 1] = e.y | ((unsigned)c << 14);
        }
        bool two = false;  // some bucket of this texel holds two pixels
#pragma unroll
        for (int c = 0; c < 4; ++c) two = two || key[2 * c + 1] != 0xFFFFFFFFu;
        if (__any(two)) {
            sort8(key);
        } else {  // one pixel per bucket in the whole wave (no magnification): 4 keys
            sort4(key[0], key[2], key[4], key[6]);
            key[1] = key[2];
            key[2] = key[4];
            key[3] = key[6];
            key[4] = key[5] = key[6] = key[7] = 0xFFFFFFFFu;
        }
        // Valid keys sort first.  A batch of 4 is branch-free and select-free: an invalid key
        // (~0) reads the zero slot kGCap (weight 0, d sample 0), and adding its +-0 leaves the sum's
        // bits unchanged -- a sum started at +0 is never -0 under round-to-nearest (x + -x and
        // +0 + -0 both give +0), and inf / NaN stay as they are.  The second batch (5+
        // contributors) is a wave-uniform branch.
        auto batch = [&](int k0) {
            float w[4];
            float4 d[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const bool v = key[k0 + k] != 0xFFFFFFFFu;
                const int q = v ? (int)(key[k0 + k] & 0x7FF) : kGCap;  // staged index: bits 0-10 (kGCap <= 2048)
                w[k] = staged_weight<FRAC>(s_w, (int)((key[k0 + k] >> 14) & 3u), q);  // corner bits 14-15
                d[k] = s_ds[q];
                hits += v ? 1u : 0u;
            }
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                acc[0] = acc[0] + w[k] * d[k].x;
                acc[1] = acc[1] + w[k] * d[k].y;
                acc[2] = acc[2] + w[k] * d[k].z;
                acc[3] = acc[3] + w[k] * d[k].w;
            }
        };
        batch(0);
        if (__any(key[4] != 0xFFFFFFFFu)) batch(4);
    } else if (tin) {
        // window scan: the inverse image of the texels [tx-1, tx+1] x [ty-1, ty+1] whose samples
        // have this texel as a tap, candidates in pixel order, the hits of one 8-pixel chunk
        // collected in a mask (bit corner*8 + pixel%8) and added in bit order
        const float* iv = ws.inv + (int64_t)p * 12;
        float m[9];
#pragma unroll
        for (int k = 0; k < 9; ++k) m[k] = iv[k];
        int wx0 = 0, wx1 = -1, wy0 = 0, wy1 = -1;
        float a0 = __builtin_inff(), a1 = -__builtin_inff(), b0 = __builtin_inff(), b1 = -__builtin_inff();
        bool lbad = false;
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            float xx, yy;
            const bool okc = inv_map(m, (float)(tx + ((c & 1) ? 1 : -1)), (float)(ty + ((c & 2) ? 1 : -1)), xx, yy);
            lbad = lbad || !okc;
            a0 = __builtin_fminf(a0, xx);
            a1 = __builtin_fmaxf(a1, xx);
            b0 = __builtin_fminf(b0, yy);
            b1 = __builtin_fmaxf(b1, yy);
        }
        if (!lbad) {
            pix_range(a0, a1, margin, bx0, bx1, wx0, wx1);
            pix_range(b0, b1, margin, by0, by1, wy0, wy1);
            // a wrapping 8-pixel chunk must not have window pixels in two rows: the per-row
            // flush below would split its order
            if ((g.W & 7) && wy1 > wy0 && wx1 >= g.W - 7 && wx0 <= 6) lbad = true;
        }
        if (lbad) {
            unsafe = true;
            wy1 = wy0 - 1;
        }
        const int ya = max(wy0, ra), yb = min(wy1, rb - 1);
        for (int yy = ya; yy <= yb; ++yy) {
            const int rowbase = (yy - ra) * bw - bx0;  // staged index of pixel (x, yy): rowbase + x
            const int pixrow = yy * g.W;
            int cur = -1;     // 8-pixel chunk (pixel / 8) of the hits in `msk`
            unsigned msk = 0;
            auto flush = [&]() {
                while (msk) {
                    const int b = __builtin_ctz(msk);
                    msk &= msk - 1;
                    const int idx = rowbase + (cur * kGridVec + (b & 7) - pixrow);
                    const float4 d = s_ds[idx];
                    const float w = staged_weight<FRAC>(s_w, b >> 3, idx);  // corner b >> 3
                    acc[0] = acc[0] + w * d.x;
                    acc[1] = acc[1] + w * d.y;
                    acc[2] = acc[2] + w * d.z;
                    acc[3] = acc[3] + w * d.w;
                    ++hits;
                }
            };
            for (int xx = wx0; xx <= wx1; ++xx) {
                const int code = s_code[rowbase + xx];
                const int dd = bt - code;  // 0: nw tap, 1: ne, TB: sw, TB+1: se
                const int c = code < 0 ? -1 : dd == 0 ? 0 : dd == 1 ? 1 : dd == TB ? 2 : dd == TB + 1 ? 3 : -1;
                if (c >= 0) {
                    const int px = pixrow + xx;
                    if ((px >> 3) != cur) {
                        flush();
                        cur = px >> 3;
                    }
                    msk |= 1u << (c * 8 + (px & 7));
                }
            }
            flush();
        }
    }
}

// Grid: (texel tiles) x (groups of kGPl planes), XCD-aware (neighbouring tiles of one
// plane group, whose pixel boxes overlap, share an XCD's L2).  The d-sample contribution
// of pixel q to texel t: weight(corner) * d s_q, added in key order from +0.  Per plane and
// pass: one staging pass (gather_stage_pass) by all 4 waves, a barrier, one texel pass
// (gather_texel_pass).  A texel's kGPl planes leave as one 16*kGPl-B run.
// Planes [p_lo, p_lo + np) (a plane group of mpiv_render_backward; p_lo a multiple of kGPl).
__device__ __forceinline__ void bwd_check_wave(BwdWs& ws, int force, int keep_abort, int l);

// Workspace flag words of the launch-folded schedule (round 6): the gather's and the fallback's
// block-exit counters (zeroed with the pair counters, reset by the last block).
constexpr int kFlagGatherDone = 8, kFlagFallbackExit = 9;

// The last block of a grid to get here returns true (block-uniform), and the device-scope atomics
// every block issued before it (the gather's pair counts) have been performed when it reads them with
// device-scope atomic loads.  No release fence: on gfx950 an agent-scope release writes back the XCD's
// L2 (the d MPI the gather just wrote), which at one fence per block cost 3x the backward (measured,
// profiles/r06_bwd_fold.json).  Instead each wave waits until its own vector memory operations are
// acknowledged (s_waitcnt vmcnt(0): device-scope atomics are acknowledged once performed) before the
// block's barrier, and the counter is a relaxed device-scope atomic.  A count read too early could
// only be smaller, which sends the view to the (bit-exact) fallback -- never a wrong gradient.
// s_flag: an int of the caller's LDS that is free by now (no extra LDS per block).
__device__ __forceinline__ bool last_block_in(int* ctr, int* s_flag) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        const unsigned prev = __hip_atomic_fetch_add(reinterpret_cast<unsigned*>(ctr), 1u, __ATOMIC_RELAXED,
                                                     __HIP_MEMORY_SCOPE_AGENT);
        const int last = prev == gridDim.x - 1;
        if (last) __hip_atomic_store(ctr, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // for the next launch
        *s_flag = last;
    }
    __syncthreads();
    return __builtin_amdgcn_readfirstlane(*s_flag) != 0;
}

// CHECK (round 6, the single-group schedule): the pair-count check (bwd_check_kernel's) runs in
// the last gather block to finish instead of a launch of its own.
template <bool CHECK = false>
__global__ __launch_bounds__(kGThreads, MPIV_GLB) void bwd_gather_kernel(RenderGeom g, const float* __restrict__ homs, BwdWs ws,
                                                         float4* __restrict__ dmpi, float margin, int p_lo, int np) {
    __shared__ int s_code[kGCap];                    // local nw-tap bucket of the staged pixel, -1 = none
    __shared__ float s_w[(MPIV_GFRAC ? 2 : 4) * kGWP];  // its bilinear weights, corner-major (kGWP), or
                                                        // (MPIV_GFRAC) its fractions; [kGCap] = 0
    __shared__ float4 s_ds[kGCap + 1];               // its d sample; [kGCap] = 0
    __shared__ unsigned s_ent[2][2 * kGNB];          // bucket lists (2 slots, ~0 = free), by pass parity
    __shared__ int s_ovf[2];                         // a list overflowed in this pass
    constexpr int TB = kGTB;
    const int tiles_x = (g.W + kGTW - 1) / kGTW;
    const int ntiles = tiles_x * ((g.H + kGTY - 1) / kGTY);
    const int lb = xcd_logical_block(blockIdx.x, gridDim.x);
    const int ngroups = (np + kGPl - 1) / kGPl;  // plane groups fastest: the blocks writing one texel's
    const int tile = lb / ngroups, p0 = p_lo + (lb % ngroups) * kGPl;  // gradient line run together
    const int p_end = p_lo + np;  // never past the group, whatever kGPl
    const int tx0 = (tile % tiles_x) * kGTW, ty0 = (tile / tiles_x) * kGTY;
    const int tx = tx0 + (threadIdx.x & (kWave - 1));
    int ty[kGTR], bt[kGTR];  // this thread's texel rows (kGTR independent texel sums per pass)
    bool tin[kGTR];
#pragma unroll
    for (int r = 0; r < kGTR; ++r) {
        ty[r] = ty0 + (int)(threadIdx.x >> 6) + r * kGTH;
        tin[r] = tx < g.W && ty[r] < g.H;
        bt[r] = (ty[r] - ty0 + 1) * TB + (tx - tx0 + 1);  // bucket of the texel as an nw tap
    }
    for (int b = threadIdx.x; b < 4 * kGNB; b += kGThreads) (&s_ent[0][0])[b] = ~0u;
    if (threadIdx.x < 2) s_ovf[threadIdx.x] = 0;
    if (threadIdx.x < (MPIV_GFRAC ? 2 : 4)) s_w[threadIdx.x * kGWP + kGCap] = 0.0f;  // FRAC: weight 1 x d sample 0
    if (threadIdx.x == 0) s_ds[kGCap] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    int par = 0;
    unsigned hits = 0;    // (texel, contributor) pairs found by this thread
    bool unsafe = false;  // a plane this block could not order (the view goes to the fallback)
    f32x4 acc[kGTR][kGPl];
#if MPIV_GPF2
    // A/B: each pass's d samples are loaded into registers during the previous pass's texel phase
    // (kGSI per thread, 12 VGPRs: the kernel stays at 4 waves/SIMD), so staging never waits on HBM
#pragma unroll
    for (int jj = 0; jj < kGPl; ++jj)
#pragma unroll
        for (int r = 0; r < kGTR; ++r) acc[r][jj] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
    int4 bxs[kGPl];
#pragma unroll
    for (int jj = 0; jj < kGPl; ++jj) {
        bxs[jj] = p0 + jj < p_end ? ws.box[(int64_t)(p0 + jj) * ntiles + tile] : make_int4(0, -1, 0, -1);
        if (bxs[jj].x == -2) {  // this block cannot gather the plane: the check sends the view to the fallback
            unsafe = true;
            bxs[jj] = make_int4(0, -1, 0, -1);
        }
    }
    auto box = [&](int jj) {  // static selects + readfirstlane: block-uniform scalars
        int4 b = make_int4(0, -1, 0, -1);
#pragma unroll
        for (int k = 0; k < kGPl; ++k)
            if (k == jj) b = bxs[k];
        return make_int4(__builtin_amdgcn_readfirstlane(b.x), __builtin_amdgcn_readfirstlane(b.y),
                         __builtin_amdgcn_readfirstlane(b.z), __builtin_amdgcn_readfirstlane(b.w));
    };
    auto first_from = [&](int jj, int& ra) {
        for (; jj < kGPl; ++jj) {
            const int4 b = box(jj);
            if (b.y >= b.x && (b.w & ~kBoxProven) >= b.z) break;
        }
        ra = jj < kGPl ? box(jj).z : 0;
        return jj;
    };
    const int64_t HWg = (int64_t)g.H * g.W;
    f32x4 pre[kGSI];
    auto load = [&](int jj, int ra) {
        if (jj >= kGPl) return;
        const int4 b = box(jj);
        const int bw = b.y - b.x + 1;
        const int rb = min((b.w & ~kBoxProven) + 1, ra + kGCap / bw);
        const int np = (rb - ra) * bw;
        const __amdgpu_buffer_rsrc_t rds = make_rsrc(ds_plane(ws, p0 + jj, HWg), (int)(HWg * 16));
        const float rbw = 1.0f / (float)bw;
#pragma unroll
        for (int i = 0; i < kGSI; ++i) {
            const int q = (int)threadIdx.x + i * kGThreads;
            const int r = (int)(((float)q + 0.5f) * rbw);
            const int off = q < np ? ((ra + r) * g.W + b.x + (q - r * bw)) * 16 : kOOB;
            pre[i] = llvm_raw_buffer_load_v4f32(rds, off, 0, 0);
        }
    };
    int ra = 0;
    int jj = first_from(0, ra);
    load(jj, ra);
    while (jj < kGPl) {
        const int4 b = box(jj);
        const int bx0 = b.x, bx1 = b.y, by0 = b.z, by1 = b.w & ~kBoxProven;
        const int bw = bx1 - bx0 + 1;
        const int rb = min(by1 + 1, ra + kGCap / bw);
        int ra_n = rb, jj_n = jj;
        if (ra_n > by1) jj_n = first_from(jj + 1, ra_n);
        const int p = p0 + jj;
        __syncthreads();  // the previous pass's readers are done
        gather_stage_pass<true, true, MPIV_GFRAC>(g, ws, homs + (int64_t)p * 9, p, (b.w & kBoxProven) != 0, (int)threadIdx.x, tx0,
                                      ty0, bx0, bw, ra, rb, s_code, s_w, s_ds, s_ent[par], &s_ovf[par], pre);
        for (int bb = threadIdx.x; bb < 2 * kGNB; bb += kGThreads) s_ent[par ^ 1][bb] = ~0u;  // for the next pass
        if (threadIdx.x == 0) s_ovf[par ^ 1] = 0;
        __syncthreads();
        load(jj_n, ra_n);  // the next pass's d samples, in flight during this texel phase
        const bool ovf = s_ovf[par] != 0;
#pragma unroll
        for (int k = 0; k < kGPl; ++k)
            if (k == jj)
#pragma unroll
                for (int r = 0; r < kGTR; ++r)
                    gather_texel_pass<MPIV_GFRAC>(g, ws, p, margin, tx, ty[r], bt[r], tin[r], ovf, s_ent[par], s_code,
                                                  s_w, s_ds, bx0, bx1, by0, by1, ra, rb, acc[r][k], hits, unsafe);
        par ^= 1;
        jj = jj_n;
        ra = ra_n;
    }
#else
#pragma unroll
    for (int jj = 0; jj < kGPl; ++jj) {
#pragma unroll
        for (int r = 0; r < kGTR; ++r) acc[r][jj] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
        const int p = p0 + jj;
        if (p >= p_end) continue;  // block-uniform
        const int4 bx = ws.box[(int64_t)p * ntiles + tile];  // bwd_box_kernel
        const int bx0 = bx.x, bx1 = bx.y, by0 = bx.z, by1 = bx.w & ~kBoxProven;
        const bool proven = (bx.w & kBoxProven) != 0;
        if (bx0 == -2) {  // this block cannot gather the plane: the check sends the view to the fallback
            unsafe = true;
            continue;
        }
        const int bw = bx1 - bx0 + 1, bh = by1 - by0 + 1;
        if (bw <= 0 || bh <= 0) continue;  // no pixel samples the tile: zero gradient (counted)
        const int rpp = kGCap / bw;  // box rows per pass
        const float* hp = homs + (int64_t)p * 9;
        for (int ra = by0; ra <= by1; ra += rpp) {
            const int rb = min(by1 + 1, ra + rpp);
            __syncthreads();  // the previous pass's readers are done
            gather_stage_pass<true, false, MPIV_GFRAC>(g, ws, hp, p, proven, (int)threadIdx.x, tx0, ty0, bx0, bw, ra,
                                                       rb, s_code, s_w, s_ds, s_ent[par], &s_ovf[par]);
            for (int b = threadIdx.x; b < 2 * kGNB; b += kGThreads) s_ent[par ^ 1][b] = ~0u;  // for the next pass
            if (threadIdx.x == 0) s_ovf[par ^ 1] = 0;
            __syncthreads();
            // block-uniform: a scalar branch, not an exec-mask split per texel (round 5, fewer scalar instructions)
            const bool ovf = __builtin_amdgcn_readfirstlane(s_ovf[par]) != 0;
#pragma unroll
            for (int r = 0; r < kGTR; ++r)
                gather_texel_pass<MPIV_GFRAC>(g, ws, p, margin, tx, ty[r], bt[r], tin[r], ovf, s_ent[par], s_code, s_w,
                                              s_ds, bx0, bx1, by0, by1, ra, rb, acc[r][jj], hits, unsafe);
            par ^= 1;
        }
    }
#endif
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) hits += __shfl_xor(hits, off);
    const unsigned long long tot = (unsigned long long)hits + (__any(unsafe) ? kUnsafe : 0ull);
    if ((threadIdx.x & (kWave - 1)) == 0 && tot) atomicAdd(&ws.found[blockIdx.x % kCtrSlots], tot);
#pragma unroll
    for (int r = 0; r < kGTR; ++r) {
        if (tin[r]) {  // the texel's kGPl planes: one 16*kGPl-B run
            float4* o = dmpi + ((int64_t)ty[r] * g.W + tx) * g.P + p0;
#pragma unroll
            for (int jj = 0; jj < kGPl; ++jj)
                if (p0 + jj < p_end) {
                    if (MPIV_BWD_NTOUT)  // A/B: d MPI past the caches (written once, never re-read here)
                        __builtin_nontemporal_store(f32x4{acc[r][jj][0], acc[r][jj][1], acc[r][jj][2], acc[r][jj][3]},
                                                    reinterpret_cast<f32x4*>(o + jj));
                    else
                        bwd_store(o + jj, make_float4(acc[r][jj][0], acc[r][jj][1], acc[r][jj][2], acc[r][jj][3]));
                }
        }
    }
    if (CHECK && last_block_in(ws.flag + kFlagGatherDone, &s_ovf[0]) && threadIdx.x < kWave)
        bwd_check_wave(ws, 0, 0, threadIdx.x);
}

#if MPIV_AB && MPIV_GTR == 1  // A/B variants of the gather (libmpiv_ab.so, one texel row per wave): measured slower, DESIGN.md §8
// ---- 2'. gather with the d samples streamed into LDS one pass ahead (bwd_gather=3) ------
// bwd_gather_kernel loads a pass's d samples in its staging phase and waits for them there;
// its texel phase issues no memory traffic, so a block's loads are in flight only part of the
// time (r03: 0.82 ms of memory phase alone, +0.8 ms with the texel phase).  Here the d samples
// of pass i+1 go from HBM straight into LDS (buffer_load_dwordx4 ... lds, no VGPRs) while pass
// i is staged and summed, so every block keeps one whole pass of loads in flight.  Only the
// fractions are staged (the texel pass forms each corner's weight with the same products), so
// a block needs 38 KiB of LDS: 4 blocks per CU.  The passes, positions, bucket lists, sums and
// counts are bwd_gather_kernel's: the gradient is bit-identical.
//
// Protocol (one barrier pair per pass, as bwd_gather_kernel): every wave issues exactly kGDF
// DMA instructions per pass (lanes past the pass's pixels get the out-of-range offset, which
// writes +0 into the buffer's tail -- the zero slot kGCap included); at the top of pass i a
// barrier retires pass i-1's texel phase, pass i+1's fill goes into the other buffer, pass i
// is staged, each wave waits for its own fills of pass i (vmcnt(kGDF): the younger kGDF are
// pass i+1's) and a barrier publishes them.  The DMA is inline asm (hipcc cannot tell which
// LDS bytes a DMA writes and would drain vmcnt(0) before every ds_read).
constexpr int kGDF = (kGCap + kGThreads - 1) / kGThreads;  // DMA instructions per wave and pass
constexpr int kGDS = kGDF * kGThreads;                     // staged slots per buffer (> kGCap)
static_assert(kGTR == 1 && kGThreads == 4 * kWave && kGDS > kGCap, "the fill covers every staged slot and the zero slot");

__device__ __forceinline__ void gather_dma16(__amdgpu_buffer_rsrc_t r, int voff, unsigned lds) {
    asm volatile("s_mov_b32 m0, %2\n\tbuffer_load_dwordx4 %0, %1, 0 offen lds" ::"v"(voff), "s"(r), "s"(lds)
                 : "memory", "m0");
}

__global__ __launch_bounds__(kGThreads, 4) void bwd_gather_dma_kernel(RenderGeom g, const float* __restrict__ homs,
                                                                      BwdWs ws, float4* __restrict__ dmpi,
                                                                      float margin) {
    __shared__ int s_code[kGCap];
    __shared__ float s_w[2 * kGWP];                               // fractions wx, wy; [kGCap] = 0
    __shared__ __attribute__((aligned(16))) float4 s_ds[2][kGDS];  // d samples by pass parity
    __shared__ unsigned s_ent[2][2 * kGNB];
    __shared__ int s_ovf[2];
    const int tiles_x = (g.W + kGTW - 1) / kGTW;
    const int ntiles = tiles_x * ((g.H + kGTH - 1) / kGTH);
    const int lb = xcd_logical_block(blockIdx.x, gridDim.x);
    const int ngroups = (g.P + kGPl - 1) / kGPl;
    const int tile = lb / ngroups, p0 = (lb % ngroups) * kGPl;
    const int tx0 = (tile % tiles_x) * kGTW, ty0 = (tile / tiles_x) * kGTH;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & (kWave - 1);
    const int tx = tx0 + lane, ty = ty0 + wave;
    const bool tin = tx < g.W && ty < g.H;
    const int bt = (ty - ty0 + 1) * kGTB + (tx - tx0 + 1);
    const int64_t HW = (int64_t)g.H * g.W;
    for (int b = threadIdx.x; b < 4 * kGNB; b += kGThreads) (&s_ent[0][0])[b] = ~0u;
    if (threadIdx.x < 2) s_ovf[threadIdx.x] = 0;
    if (threadIdx.x < 2) s_w[threadIdx.x * kGWP + kGCap] = 0.0f;
    unsigned hits = 0;
    bool unsafe = false;
    // the block's planes: boxes (bwd_box_kernel); a box the block cannot gather makes the view unsafe
    int4 bxs[kGPl];
#pragma unroll
    for (int jj = 0; jj < kGPl; ++jj) {
        bxs[jj] = p0 + jj < g.P ? ws.box[(int64_t)(p0 + jj) * ntiles + tile] : make_int4(0, -1, 0, -1);
        if (bxs[jj].x == -2) {
            unsafe = true;
            bxs[jj] = make_int4(0, -1, 0, -1);
        }
    }
    // passes: (plane jj, first box row ra); jj == kGPl ends.  box(jj): static selects, then
    // readfirstlane (block-uniform values: the buffer descriptor and M0 need SGPRs)
    auto box = [&](int jj) {
        int4 b = make_int4(0, -1, 0, -1);
#pragma unroll
        for (int k = 0; k < kGPl; ++k)
            if (k == jj) b = bxs[k];
        return make_int4(__builtin_amdgcn_readfirstlane(b.x), __builtin_amdgcn_readfirstlane(b.y),
                         __builtin_amdgcn_readfirstlane(b.z), __builtin_amdgcn_readfirstlane(b.w));
    };
    auto rows_per_pass = [&](const int4& b) { return kGCap / (b.y - b.x + 1); };
    auto first_from = [&](int jj, int& ra) {
        for (; jj < kGPl; ++jj) {
            const int4 b = box(jj);
            if (b.y >= b.x && (b.w & ~kBoxProven) >= b.z) break;
        }
        ra = jj < kGPl ? box(jj).z : 0;
        return jj;
    };
    auto fill = [&](int jj, int ra, int buf) {  // kGDF DMA instructions of this wave
        int np = 0, bw = 1, bx0 = 0;
        const float* base = reinterpret_cast<const float*>(ds_plane(ws, 0, 0));
        if (jj < kGPl) {
            const int4 b = box(jj);
            bx0 = b.x;
            bw = b.y - bx0 + 1;
            const int rb = min((b.w & ~kBoxProven) + 1, ra + rows_per_pass(b));
            np = (rb - ra) * bw;
            base = reinterpret_cast<const float*>(ds_plane(ws, p0 + jj, HW));
        }
        const __amdgpu_buffer_rsrc_t r = make_rsrc(base, (int)(HW * 16));
        const float rbw = 1.0f / (float)bw;
        const unsigned lds = (unsigned)(uintptr_t)&s_ds[buf][0] + (unsigned)wave * kWave * 16;
#pragma unroll
        for (int f = 0; f < kGDF; ++f) {
            const int q = (f * 4 + wave) * kWave + lane;
            const int rr = (int)(((float)q + 0.5f) * rbw);  // q / bw (gather_stage_pass)
            const int voff = q < np ? ((ra + rr) * g.W + bx0 + (q - rr * bw)) * 16 : kOOB;
            gather_dma16(r, voff, __builtin_amdgcn_readfirstlane(lds + (unsigned)(f * kGThreads * 16)));
        }
    };
    f32x4 acc[kGPl];
#pragma unroll
    for (int jj = 0; jj < kGPl; ++jj) acc[jj] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
    int ra = 0;
    int jj = first_from(0, ra);
    if (jj < kGPl) fill(jj, ra, 0);
    int par = 0;
    while (jj < kGPl) {
        const int4 bj = box(jj);
        const int by1 = bj.w & ~kBoxProven, rpp = rows_per_pass(bj);
        const int rb = min(by1 + 1, ra + rpp);
        int ra_n = rb, jj_n = jj;
        if (ra_n > by1) jj_n = first_from(jj + 1, ra_n);
        __syncthreads();  // the previous pass's texel phase is done with buffer par ^ 1 and the staging arrays
        const bool more = jj_n < kGPl;
        if (more) fill(jj_n, ra_n, par ^ 1);
        const int p = p0 + jj;
        const int bx0 = bj.x, bx1 = bj.y, by0 = bj.z;
        gather_stage_pass<false>(g, ws, homs + (int64_t)p * 9, p, (bj.w & kBoxProven) != 0, (int)threadIdx.x,
                                 tx0, ty0, bx0, bx1 - bx0 + 1, ra, rb, s_code, s_w, nullptr, s_ent[par], &s_ovf[par]);
        for (int b = threadIdx.x; b < 2 * kGNB; b += kGThreads) s_ent[par ^ 1][b] = ~0u;  // for the next pass
        if (threadIdx.x == 0) s_ovf[par ^ 1] = 0;
        if (more)
            asm volatile("s_waitcnt vmcnt(%0)" ::"n"(kGDF) : "memory");  // this pass's fills (pass i+1's are younger)
        else
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        // jj is block-uniform: the accumulator index stays static after unrolling the select
#pragma unroll
        for (int k = 0; k < kGPl; ++k)
            if (k == jj)
                gather_texel_pass<true>(g, ws, p, margin, tx, ty, bt, tin, s_ovf[par] != 0, s_ent[par], s_code, s_w,
                                        s_ds[par], bx0, bx1, by0, by1, ra, rb, acc[k], hits, unsafe);
        par ^= 1;
        jj = jj_n;
        ra = ra_n;
    }
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) hits += __shfl_xor(hits, off);
    const unsigned long long tot = (unsigned long long)hits + (__any(unsafe) ? kUnsafe : 0ull);
    if (lane == 0 && tot) atomicAdd(&ws.found[blockIdx.x % kCtrSlots], tot);
    if (tin) {
        float4* o = dmpi + ((int64_t)ty * g.W + tx) * g.P + p0;
#pragma unroll
        for (int k = 0; k < kGPl; ++k)
            if (p0 + k < g.P) o[k] = make_float4(acc[k][0], acc[k][1], acc[k][2], acc[k][3]);
    }
}


// ---- 2a'. gather with staging and texel waves (bwd_gather=2) ---------------------------
// bwd_gather_kernel alternates a memory phase (the staging pass: d-sample loads, positions)
// and a compute phase (the sorted per-texel sums) behind block barriers, and the two barely
// overlap (r03 diagnostics: 0.82 ms of memory phase alone, ~0.9 ms of texel phase on top).
// Here a block of 8 waves splits the roles: waves 0-3 stage pass i+1 into one buffer while
// waves 4-7 sum pass i from the other, one barrier per pass.  Both roles walk the same pass
// sequence (planes p0.., box row passes), the texel waves one pass behind; bucket sizes are
// triple-buffered (filled for pass i+1, read for pass i, zeroed for pass i+2).
__global__ __launch_bounds__(2 * kGThreads, MPIV_GLBS) void bwd_gather_ws_kernel(RenderGeom g,
                                                                          const float* __restrict__ homs, BwdWs ws,
                                                                          float4* __restrict__ dmpi, float margin) {
    __shared__ int s_code[2][kGCap];
    __shared__ float s_w[2][4 * kGWP];
    __shared__ float4 s_ds[2][kGCap + 1];
    __shared__ unsigned s_ent[3][2 * kGNB];
    __shared__ int s_ovf[3];
    constexpr int TB = kGTB;
    const int tiles_x = (g.W + kGTW - 1) / kGTW;
    const int ntiles = tiles_x * ((g.H + kGTH - 1) / kGTH);
    const int lb = xcd_logical_block(blockIdx.x, gridDim.x);
    const int ngroups = (g.P + kGPl - 1) / kGPl;
    const int tile = lb / ngroups, p0 = (lb % ngroups) * kGPl;
    const int tx0 = (tile % tiles_x) * kGTW, ty0 = (tile / tiles_x) * kGTH;
    const bool stager = threadIdx.x < kGThreads;  // wave-uniform
    const int t = (int)threadIdx.x & (kGThreads - 1);
    for (int b = threadIdx.x; b < 6 * kGNB; b += 2 * kGThreads) (&s_ent[0][0])[b] = ~0u;
    if (threadIdx.x < 3) s_ovf[threadIdx.x] = 0;
    if (threadIdx.x < 8) s_w[threadIdx.x >> 2][(threadIdx.x & 3) * kGWP + kGCap] = 0.0f;
    if (threadIdx.x < 2) s_ds[threadIdx.x][kGCap] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    // the pass sequence: (plane jj, box rows [ra, rb)); seek() finds the first pass at or after
    // (jj, ra) (ra = INT_MIN: plane jj's first), skipping planes without pixels; the texel role
    // notes planes it cannot order (bad boxes) as it passes them
    struct Pass {
        int jj, bx0, bx1, by0, by1, ra, rb;
        bool proven;
    };
    bool unsafe = false;
    auto seek = [&](int jj, int ra, Pass& ps) -> bool {
        for (; jj < kGPl; ++jj, ra = INT_MIN) {
            const int p = p0 + jj;
            if (p >= g.P) return false;
            const int4 bx = ws.box[(int64_t)p * ntiles + tile];  // bwd_box_kernel
            if (bx.x == -2) {
                if (ra == INT_MIN) unsafe = true;
                continue;
            }
            const int by1 = bx.w & ~kBoxProven;
            const int bw = bx.y - bx.x + 1;
            const int start = ra == INT_MIN ? bx.z : ra;
            if (bw <= 0 || by1 < bx.z || start > by1) continue;
            ps.jj = jj;
            ps.bx0 = bx.x;
            ps.bx1 = bx.y;
            ps.by0 = bx.z;
            ps.by1 = by1;
            ps.ra = start;
            ps.rb = min(by1 + 1, start + kGCap / bw);
            ps.proven = (bx.w & kBoxProven) != 0;
            return true;
        }
        return false;
    };
    __syncthreads();  // counts zeroed
    Pass cur;
    bool have = seek(0, INT_MIN, cur);
    if (stager) {
        if (have)
            gather_stage_pass(g, ws, homs + (int64_t)(p0 + cur.jj) * 9, p0 + cur.jj, cur.proven, t, tx0, ty0, cur.bx0,
                              cur.bx1 - cur.bx0 + 1, cur.ra, cur.rb, s_code[0], s_w[0], s_ds[0], s_ent[0],
                              &s_ovf[0]);
        __syncthreads();
        for (int i = 0; have; ++i) {
            Pass nxt;
            have = seek(cur.jj, cur.rb, nxt);
            if (have)
                gather_stage_pass(g, ws, homs + (int64_t)(p0 + nxt.jj) * 9, p0 + nxt.jj, nxt.proven, t, tx0, ty0,
                                  nxt.bx0, nxt.bx1 - nxt.bx0 + 1, nxt.ra, nxt.rb, s_code[(i + 1) & 1],
                                  s_w[(i + 1) & 1], s_ds[(i + 1) & 1], s_ent[(i + 1) % 3], &s_ovf[(i + 1) % 3]);
            for (int b = t; b < 2 * kGNB; b += kGThreads) s_ent[(i + 2) % 3][b] = ~0u;  // for pass i + 2
            if (t == 0) s_ovf[(i + 2) % 3] = 0;
            __syncthreads();
            cur = nxt;
        }
        return;  // every barrier of the texel waves has been matched
    }
    // texel waves: planes unrolled (static accumulator per plane), passes in sequence order
    const int tx = tx0 + (t & (kWave - 1)), ty = ty0 + (t >> 6);
    const bool tin = tx < g.W && ty < g.H;
    const int bt = (ty - ty0 + 1) * TB + (tx - tx0 + 1);
    unsigned hits = 0;
    f32x4 acc[kGPl];
#pragma unroll
    for (int jj = 0; jj < kGPl; ++jj) acc[jj] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
    __syncthreads();  // pass 0 staged
    int i = 0;
#pragma unroll
    for (int jj = 0; jj < kGPl; ++jj) {
        while (have && cur.jj == jj) {
            gather_texel_pass(g, ws, p0 + jj, margin, tx, ty, bt, tin, s_ovf[i % 3] != 0, s_ent[i % 3], s_code[i & 1],
                              s_w[i & 1], s_ds[i & 1], cur.bx0, cur.bx1, cur.by0, cur.by1, cur.ra, cur.rb, acc[jj],
                              hits, unsafe);
            Pass nxt;
            have = seek(cur.jj, cur.rb, nxt);
            __syncthreads();  // pass i + 1 staged; pass i's buffers free
            cur = nxt;
            ++i;
        }
    }
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) hits += __shfl_xor(hits, off);
    const unsigned long long tot = (unsigned long long)hits + (__any(unsafe) ? kUnsafe : 0ull);
    if ((t & (kWave - 1)) == 0 && tot) atomicAdd(&ws.found[blockIdx.x % kCtrSlots], tot);
    if (tin) {
        float4* o = dmpi + ((int64_t)ty * g.W + tx) * g.P + p0;
#pragma unroll
        for (int jj = 0; jj < kGPl; ++jj)
            if (p0 + jj < g.P) o[jj] = make_float4(acc[jj][0], acc[jj][1], acc[jj][2], acc[jj][3]);
    }
}

// ---- 2b. gather, one texel row per wave (bwd_gather=1) ---------------------------------
// The same per-texel sums and keys as bwd_gather_kernel, but every wave works alone on its
// 64-texel row: it maps its own bucket region [tx0-1, tx0+63] x [ty-1, ty] (nw taps) back to a
// box of pixels, stages their sample positions in wave-private LDS and reads the d samples of
// the contributors it finds straight from memory -- no block barriers, so the waves of a CU
// drift apart and one wave's memory round trip hides behind another's arithmetic.
constexpr int kWCap = 256;              // staged pixels per wave pass
constexpr int kWNB = kGTB * 2;          // bucket rows: nw-tap y = ty - 1, ty
__device__ __forceinline__ void wave_lds_fence() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

#ifndef MPIV_GLBW
#define MPIV_GLBW 6
#endif
__global__ __launch_bounds__(256, MPIV_GLBW) void bwd_gather_wave_kernel(RenderGeom g, const float* __restrict__ homs,
                                                                   BwdWs ws, float4* __restrict__ dmpi, float margin) {
    __shared__ int s_code_a[4][kWCap];   // local nw-tap bucket of the staged pixel, -1 = none
    __shared__ float2 s_fr_a[4][kWCap];  // its bilinear fractions
    __shared__ int s_pix_a[4][kWCap];    // its pixel index (y*W + x)
    __shared__ uint2 s_bent_a[4][kWNB];  // bucket lists (kGBCap entries)
    __shared__ int s_bcnt_a[4][kWNB];    // bucket sizes
    constexpr int TB = kGTB;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & (kWave - 1);
    int* s_code = s_code_a[wave];
    float2* s_fr = s_fr_a[wave];
    int* s_pix = s_pix_a[wave];
    uint2* s_bent = s_bent_a[wave];
    int* s_bcnt = s_bcnt_a[wave];
    const int tiles_x = (g.W + kGTW - 1) / kGTW;
    const int lb = xcd_logical_block(blockIdx.x, gridDim.x);
    const int ngroups = (g.P + kGPl - 1) / kGPl;
    const int tile = lb / ngroups, p0 = (lb % ngroups) * kGPl;
    const int tx0 = (tile % tiles_x) * kGTW, ty = (tile / tiles_x) * kGTH + wave;
    if (ty >= g.H) return;  // whole wave; no block barrier anywhere below
    const int tx = tx0 + lane;
    const bool tin = tx < g.W;
    const int64_t HW = (int64_t)g.H * g.W;
    const int bt = TB + lane + 1;  // bucket of the texel as an nw tap (row 1: nw-tap y = ty)
    for (int b = lane; b < kWNB; b += kWave) s_bcnt[b] = 0;
    unsigned hits = 0;
    bool unsafe = false;
    f32x4 acc[kGPl];
#pragma unroll
    for (int jj = 0; jj < kGPl; ++jj) {
        acc[jj] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
        const int p = p0 + jj;
        if (p >= g.P) continue;  // wave-uniform
        // the box of pixels whose samples can have their nw tap in the bucket region:
        // samples in [tx0-1, tx0+kGTW) x [ty-1, ty+1), inverse image of the corners + margin
        const float* iv = ws.inv + (int64_t)p * 12;
        bool bad = iv[9] == 0.0f;
        float xmn = __builtin_inff(), xmx = -__builtin_inff(), ymn = __builtin_inff(), ymx = -__builtin_inff();
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            float mb[9];
#pragma unroll
            for (int k = 0; k < 9; ++k) mb[k] = iv[k];
            float xx, yy;
            const bool okc = inv_map(mb, (float)((c & 1) ? tx0 + kGTW : tx0 - 1), (float)((c & 2) ? ty + 1 : ty - 1), xx, yy);
            bad = bad || !okc;
            xmn = __builtin_fminf(xmn, xx);
            xmx = __builtin_fmaxf(xmx, xx);
            ymn = __builtin_fminf(ymn, yy);
            ymx = __builtin_fmaxf(ymx, yy);
        }
        int bx0 = 0, bx1 = -1, by0 = 0, by1 = -1;
        if (!bad) {
            pix_range(xmn, xmx, margin, 0, g.W - 1, bx0, bx1);
            pix_range(ymn, ymx, margin, 0, g.H - 1, by0, by1);
            const int bw = bx1 - bx0 + 1, bh = by1 - by0 + 1;
            if (bw > 0 && bh > 0) {
                const int rpp = bw <= kWCap ? kWCap / bw : 1;
                bad = bw > kWCap || (int64_t)bw * bh > 64 * kWCap ||
                      (bh > rpp && (g.W & 7) && bx0 <= 6 && bx1 >= g.W - 7);
            }
        }
        if (bad) {  // this wave cannot gather the plane: the check sends the view to the fallback
            unsafe = true;
            continue;
        }
        const int bw = bx1 - bx0 + 1, bh = by1 - by0 + 1;
        if (bw <= 0 || bh <= 0) continue;  // no pixel samples the row: zero gradient (counted)
        const float* hp = homs + (int64_t)p * 9;
        const bool proven = div2_rect_safe(hp, (float)bx0, (float)bx1, (float)by0, (float)by1);
        const int rpp = kWCap / bw;
        const float4* dsp = ds_plane(ws, p, HW);
        for (int ra = by0; ra <= by1; ra += rpp) {
            const int rb = min(by1 + 1, ra + rpp);
            const int np = (rb - ra) * bw;
            const int gbase = (ra * g.W) >> 3;
            bool ovf = (int64_t)(rb - ra + 1) * g.W >= ((int64_t)1 << 19);  // keys hold chunk - gbase in 16 bits
            const float rbw = 1.0f / (float)bw;
            for (int q = lane; q < np; q += kWave) {
                const int r = (int)(((float)q + 0.5f) * rbw);  // q / bw
                const int yy = ra + r, xx = bx0 + (q - r * bw);
                float px, py;
                if (proven)
                    render_pos_fast<false>(hp, (float)xx, (float)yy, g, px, py);
                else
                    render_pos<true>(hp, (float)xx, (float)yy, g, px, py);
                const float fx0 = floorf(px), fy0 = floorf(py);
                const float lx = fx0 - (float)(tx0 - 1), ly = fy0 - (float)(ty - 1);
                const bool in = lx >= 0.0f && lx <= (float)kGTW && ly >= 0.0f && ly <= 1.0f;
                const int code = in ? (int)ly * TB + (int)lx : -1;
                const int pix = yy * g.W + xx;
                s_code[q] = code;
                if (in) {
                    s_fr[q] = make_float2(px - fx0, py - fy0);
                    s_pix[q] = pix;
                    const unsigned e = ((unsigned)((pix >> 3) - gbase) << 16) | ((unsigned)(pix & 7) << 11) | (unsigned)q;
                    const int slot = atomicAdd(&s_bcnt[code], 1);
                    if (slot < kGBCap)
                        (slot == 0 ? s_bent[code].x : s_bent[code].y) = e;
                    else
                        ovf = true;
                }
            }
            wave_lds_fence();
            ovf = __any(ovf);
            if (tin && !ovf) {
                unsigned key[8];
#pragma unroll
                for (int c = 0; c < 4; ++c) {
                    const int b = bt - (c & 1) - (c >> 1) * TB;
                    const int n = s_bcnt[b];
                    const uint2 e = s_bent[b];
                    key[2 * c] = n > 0 ? (e.x | ((unsigned)c << 14)) : 0xFFFFFFFFu;
                    key[2 * c + 1] = n > 1 ? (e.y | ((unsigned)c << 14)) : 0xFFFFFFFFu;
                }
                bool two = false;
#pragma unroll
                for (int c = 0; c < 4; ++c) two = two || key[2 * c + 1] != 0xFFFFFFFFu;
                if (__any(two)) {
                    sort8(key);
                } else {
                    sort4(key[0], key[2], key[4], key[6]);
                    key[1] = key[2];
                    key[2] = key[4];
                    key[3] = key[6];
                    key[4] = key[5] = key[6] = key[7] = 0xFFFFFFFFu;
                }
#pragma unroll
                for (int k0 = 0; k0 < 8; k0 += 4) {
                    if (key[k0] == 0xFFFFFFFFu) break;
                    float2 f[4];
                    float4 d[4];
#pragma unroll
                    for (int k = 0; k < 4; ++k) {
                        if (key[k0 + k] != 0xFFFFFFFFu) {
                            const int q = (int)(key[k0 + k] & 0x7FF);
                            f[k] = s_fr[q];
                            d[k] = dsp[s_pix[q]];
                        }
                    }
#pragma unroll
                    for (int k = 0; k < 4; ++k) {
                        if (key[k0 + k] != 0xFFFFFFFFu) {
                            const float wx = f[k].x, ex = 1.0f - wx;
                            const float wy = f[k].y, sy = 1.0f - wy;
                            const unsigned c = key[k0 + k] >> 14;
                            const float w = ((c & 2) ? wy : sy) * ((c & 1) ? wx : ex);
                            acc[jj][0] = acc[jj][0] + w * d[k].x;
                            acc[jj][1] = acc[jj][1] + w * d[k].y;
                            acc[jj][2] = acc[jj][2] + w * d[k].z;
                            acc[jj][3] = acc[jj][3] + w * d[k].w;
                            ++hits;
                        }
                    }
                }
            } else if (tin) {
                // window scan (magnification): bwd_gather_kernel's, on this wave's staging
                float m[9];  // the inverse map again (not kept live through the fill)
#pragma unroll
                for (int k = 0; k < 9; ++k) m[k] = iv[k];
                int wx0 = 0, wx1 = -1, wy0 = 0, wy1 = -1;
                float a0 = __builtin_inff(), a1 = -__builtin_inff(), b0 = __builtin_inff(), b1 = -__builtin_inff();
                bool lbad = false;
#pragma unroll
                for (int c = 0; c < 4; ++c) {
                    float xx, yy;
                    const bool okc = inv_map(m, (float)(tx + ((c & 1) ? 1 : -1)), (float)(ty + ((c & 2) ? 1 : -1)), xx, yy);
                    lbad = lbad || !okc;
                    a0 = __builtin_fminf(a0, xx);
                    a1 = __builtin_fmaxf(a1, xx);
                    b0 = __builtin_fminf(b0, yy);
                    b1 = __builtin_fmaxf(b1, yy);
                }
                if (!lbad) {
                    pix_range(a0, a1, margin, bx0, bx1, wx0, wx1);
                    pix_range(b0, b1, margin, by0, by1, wy0, wy1);
                    if ((g.W & 7) && wy1 > wy0 && wx1 >= g.W - 7 && wx0 <= 6) lbad = true;
                }
                if (lbad) {
                    unsafe = true;
                    wy1 = wy0 - 1;
                }
                const int ya = max(wy0, ra), yb = min(wy1, rb - 1);
                for (int yy = ya; yy <= yb; ++yy) {
                    const int rowbase = (yy - ra) * bw - bx0;
                    const int pixrow = yy * g.W;
                    int cur = -1;
                    unsigned msk = 0;
                    auto flush = [&]() {
                        while (msk) {
                            const int b = __builtin_ctz(msk);
                            msk &= msk - 1;
                            const int idx = rowbase + (cur * kGridVec + (b & 7) - pixrow);
                            const float2 f = s_fr[idx];
                            const float4 d = dsp[s_pix[idx]];
                            const float wx = f.x, ex = 1.0f - wx;
                            const float wy = f.y, sy = 1.0f - wy;
                            const int c = b >> 3;
                            const float w = ((c & 2) ? wy : sy) * ((c & 1) ? wx : ex);
                            acc[jj][0] = acc[jj][0] + w * d.x;
                            acc[jj][1] = acc[jj][1] + w * d.y;
                            acc[jj][2] = acc[jj][2] + w * d.z;
                            acc[jj][3] = acc[jj][3] + w * d.w;
                            ++hits;
                        }
                    };
                    for (int xx = wx0; xx <= wx1; ++xx) {
                        const int code = s_code[rowbase + xx];
                        const int dd = bt - code;  // 0: nw tap, 1: ne, TB: sw, TB+1: se
                        const int c = code < 0 ? -1 : dd == 0 ? 0 : dd == 1 ? 1 : dd == TB ? 2 : dd == TB + 1 ? 3 : -1;
                        if (c >= 0) {
                            const int px = pixrow + xx;
                            if ((px >> 3) != cur) {
                                flush();
                                cur = px >> 3;
                            }
                            msk |= 1u << (c * 8 + (px & 7));
                        }
                    }
                    flush();
                }
            }
            wave_lds_fence();  // every lane has read the lists before they are cleared
            for (int b = lane; b < kWNB; b += kWave) s_bcnt[b] = 0;
            wave_lds_fence();
        }
    }
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) hits += __shfl_xor(hits, off);
    const unsigned long long tot = (unsigned long long)hits + (__any(unsafe) ? kUnsafe : 0ull);
    if (lane == 0 && tot) atomicAdd(&ws.found[blockIdx.x % kCtrSlots], tot);
    if (tin) {
        float4* o = dmpi + ((int64_t)ty * g.W + tx) * g.P + p0;
#pragma unroll
        for (int jj = 0; jj < kGPl; ++jj)
            if (p0 + jj < g.P) o[jj] = make_float4(acc[jj][0], acc[jj][1], acc[jj][2], acc[jj][3]);
    }
}

#endif  // MPIV_AB

// ---- 3. check: found == truth, else the fallback runs; counters reset for the next view
// keep_abort: a later plane group of the same view (flag[3] stays set once any group aborted)
// one wave (lane l = threadIdx.x & 63): the two pair counts summed, compared and reset
__device__ __forceinline__ void bwd_check_wave(BwdWs& ws, int force, int keep_abort, int l) {
    unsigned long long t = __hip_atomic_load(&ws.truth[l], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    unsigned long long f = __hip_atomic_load(&ws.found[l], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
        t += __shfl_xor(t, off);
        f += __shfl_xor(f, off);
    }
    ws.truth[l] = 0;
    ws.found[l] = 0;
    if (l == 0) {
        ws.flag[0] = (force || t != f) ? 1 : 0;
        ws.flag[1] = 0;  // the fallback's ticket and completion counters, abort flag
        ws.flag[2] = 0;
        if (!keep_abort) ws.flag[3] = 0;
    }
}

__global__ __launch_bounds__(kWave) void bwd_check_kernel(BwdWs ws, int force, int keep_abort) {
    bwd_check_wave(ws, force, keep_abort, threadIdx.x);
}

// ---- fallback: the general bucket pipeline (runs only when flag[0] is set) -----------
// One launch per view (bwd_fallback_kernel) that returns at once while the flag is clear.
// Per chunk of ws.pc planes, kFbPhases phases: nw-tap bucket of every sample and bucket sizes,
// tile sums of the sizes, their scan (one block), the exclusive scan applied, pixel ids into
// their buckets, small buckets sorted by pixel id (large ones listed), large buckets sorted by
// a whole block each, then per texel the four buckets merged in the reference's order; one
// phase up front zeroes the sizes.  Each phase is a grid-stride loop over nblk virtual blocks.
// (A normal launch, not hipLaunchCooperativeKernel: rocprofv3's kernel tracer crashes in its
// teardown after a cooperative launch, and this one is issued on every backward.)
//
// The phases are ordered by TICKETS, not by grid barriers (round 3's schedule assumed every
// block resident, "the stream runs nothing beside it" -- RCCL kernels or another process on
// the device break that).  A block takes the next ticket t (flag[1], one
// device-scope atomic): virtual block t % nblk of phase ph = t / nblk.  It waits until the
// completion counter (flag[2]) reaches ph * nblk, runs the item and adds one to the counter.
// The counter counts items of every phase, yet reaching ph * nblk means exactly "every item of
// phases < ph is done": an item of phase q only runs after seeing the counter at >= q * nblk,
// so the completions counted before it first reaches ph * nblk all come from phases < ph,
// which hold ph * nblk items.  Tickets are taken in increasing order, so every item a waiting
// block depends on was taken earlier by a block that is running (a block that is not resident
// holds no ticket), and the holder of the lowest unfinished ticket never waits: the pipeline
// completes whatever else the device runs and however few of its blocks are resident
// (`test_backward_fallback_more_blocks_than_resident`: 20000 blocks).  A wait longer than its
// poll limit (never expected: the argument above) sets flag[3], counts the view in flag[4]
// and every block stops; bwd_poison_kernel then fills the view's gradient with NaN and
// mpiv_render_backward_status reports it -- never a plausible wrong gradient.
// A/B: bwd_fb_mode=1 runs round 3's barrier schedule (bwd_fallback_barrier_kernel, with the
// same loud abort), 2 the ticket kernel with a fixed item order.
constexpr int kFbPhases = 8;  // per plane chunk

__device__ __forceinline__ int block_exclusive_scan(int v, int* s_tmp, int& total) {
    // 256 threads: inclusive Hillis-Steele scan through LDS
    s_tmp[threadIdx.x] = v;
    __syncthreads();
    for (int off = 1; off < kScanBlock; off <<= 1) {
        const int add = threadIdx.x >= off ? s_tmp[threadIdx.x - off] : 0;
        __syncthreads();
        s_tmp[threadIdx.x] += add;
        __syncthreads();
    }
    total = s_tmp[kScanBlock - 1];
    const int incl = s_tmp[threadIdx.x];
    __syncthreads();
    return incl - v;
}

// Grid-wide barrier (the production fallback's phases): arrive = one device-scope atomic per
// block after a release fence, wait = poll the counter (flag[1], zeroed by bwd_check_kernel)
// until every block of this phase has arrived, then an acquire fence (the fences write back /
// invalidate the XCD's L2, so the next phase sees every block's stores).  The launch is sized
// so every block is resident (<= 4 per CU and the device's occupancy for it); should a wait
// still outlast poll_limit polls (blocks kept from residency by other work on the device), the
// block sets flag[3], counts the view in flag[4] and every block leaves at its next barrier:
// bwd_poison_kernel then NaN-fills the view's gradient and mpiv_render_backward_status reports
// it -- never a plausible wrong gradient.  poll_limit 0 (tests): abort at the first barrier.
__device__ __forceinline__ bool grid_barrier(int* flag, unsigned target, unsigned poll_limit, int* s_abort) {
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned* ctr = reinterpret_cast<unsigned*>(flag + 1);
        int ab = 0;
        __threadfence();
        atomicAdd(ctr, 1u);
        if (poll_limit == 0) {
            if (atomicExch(flag + 3, 1) == 0) atomicAdd(flag + 4, 1);
            ab = 1;
        }
        unsigned spins = 0;
        while (!ab && __hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
            if (__hip_atomic_load(flag + 3, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0) {
                ab = 1;
                break;
            }
            __builtin_amdgcn_s_sleep(2);
            if (++spins > poll_limit) {
                if (atomicExch(flag + 3, 1) == 0) atomicAdd(flag + 4, 1);
                ab = 1;
            }
        }
        __threadfence();
        *s_abort = ab;
    }
    __syncthreads();
    return *s_abort != 0;
}

__device__ __forceinline__ unsigned order_key(int pix, int corner) {
    return ((unsigned)(pix / kGridVec) << 5) | ((unsigned)corner << 3) | (unsigned)(pix % kGridVec);
}

#if MPIV_AB  // the round-3 schedule: phases at grid barriers over resident blocks (bwd_fb_mode=1)
template <bool FAST>
__global__ __launch_bounds__(256) void bwd_fallback_barrier_kernel(RenderGeom g, const float* __restrict__ homs, BwdWs ws,
                                                           float4* __restrict__ dmpi, unsigned poll_limit) {
    __shared__ int s_tmp[kScanBlock];
    __shared__ int s_abort;
    if (ws.flag[0] == 0) return;  // uniform over the grid: the tile gather was complete
    const int bid = blockIdx.x, nblk = gridDim.x, tid = threadIdx.x;
    unsigned phase = 0;
    // true: the pipeline aborted (a wait gave up here or in another block): every block stops
    auto sync = [&]() { return grid_barrier(ws.flag, ++phase * (unsigned)nblk, poll_limit, &s_abort); };
    const int64_t gtid = (int64_t)bid * 256 + tid, gstride = (int64_t)nblk * 256;
    const int64_t HW = (int64_t)g.H * g.W;
    const int K1 = g.W + 1;
    const int64_t K = (int64_t)(g.H + 1) * K1;
    // bucket sizes start at zero (the fill returns them to zero for the next chunk)
    for (int64_t i = gtid; i < (int64_t)ws.pc * K; i += gstride) ws.count[i] = 0;
    if (sync()) return;
    for (int pc0 = 0; pc0 < g.P; pc0 += ws.pc) {
        const int pcn = min(ws.pc, g.P - pc0);
        const int64_t nq = pcn * HW, nk = pcn * K;
        const int nb = (int)((nk + kScanTile - 1) / kScanTile);
        // nw-tap bucket of every (plane of the chunk, pixel) sample; sizes counted
        for (int64_t q = gtid; q < nq; q += gstride) {
            const int pl = (int)(q / HW);
            const int pix = (int)(q - pl * HW);
            const int y = pix / g.W, x = pix - y * g.W;
            float px, py;
            render_pos<FAST>(homs + (int64_t)(pc0 + pl) * 9, (float)x, (float)y, g, px, py);
            const float fx0 = floorf(px), fy0 = floorf(py);
            // some tap lies in the image iff the nw tap is in [-1, W-1] x [-1, H-1] (NaN: none)
            const bool in = fx0 >= -1.0f && fx0 <= (float)(g.W - 1) && fy0 >= -1.0f && fy0 <= (float)(g.H - 1);
            const int k = in ? ((int)fy0 + 1) * K1 + (int)fx0 + 1 : -1;
            ws.key[q] = k;
            if (in) atomicAdd(&ws.count[pl * K + k], 1);
        }
        if (sync()) return;
        // exclusive scan of the sizes: tile sums, their scan (block 0), per-tile apply
        for (int tb = bid; tb < nb; tb += nblk) {
            const int64_t base = (int64_t)tb * kScanTile + (int64_t)tid * kScanItems;
            int sum = 0;
            for (int i = 0; i < kScanItems; ++i)
                if (base + i < nk) sum += ws.count[base + i];
            int total;
            block_exclusive_scan(sum, s_tmp, total);
            if (tid == 0) ws.bsum[tb] = total;
        }
        if (sync()) return;
        if (bid == 0) {
            int carry = 0;
            for (int c0 = 0; c0 < nb; c0 += kScanBlock) {
                const int i = c0 + tid;
                const int v = i < nb ? ws.bsum[i] : 0;
                int total;
                const int ex = block_exclusive_scan(v, s_tmp, total);
                if (i < nb) ws.bsum[i] = carry + ex;
                carry += total;
            }
            if (tid == 0) ws.big[0] = 0;
        }
        if (sync()) return;
        for (int tb = bid; tb < nb; tb += nblk) {
            const int64_t base = (int64_t)tb * kScanTile + (int64_t)tid * kScanItems;
            int v[kScanItems];
            int sum = 0;
#pragma unroll
            for (int i = 0; i < kScanItems; ++i) {
                v[i] = base + i < nk ? ws.count[base + i] : 0;
                sum += v[i];
            }
            int total;
            int run = ws.bsum[tb] + block_exclusive_scan(sum, s_tmp, total);
#pragma unroll
            for (int i = 0; i < kScanItems; ++i) {
                if (base + i < nk) ws.offs[base + i] = run;
                run += v[i];
            }
            if (tb == nb - 1 && tid == kScanBlock - 1) ws.offs[nk] = run;  // grand total
        }
        if (sync()) return;
        // pixel ids into their buckets (atomic slot claim; sizes return to zero)
        for (int64_t q = gtid; q < nq; q += gstride) {
            const int k = ws.key[q];
            if (k < 0) continue;
            const int64_t pl = q / HW;
            const int64_t pk = pl * K + k;
            const int slot = atomicSub(&ws.count[pk], 1) - 1;
            ws.ids[ws.offs[pk] + slot] = (int)(q - pl * HW);
        }
        if (sync()) return;
        // each bucket sorted by pixel id: <= kSmallBucket ids by one thread (insertion
        // sort), larger ones (minification, degenerate homographies) listed for a block
        for (int64_t pk = gtid; pk < nk; pk += gstride) {
            const int b = ws.offs[pk], e = ws.offs[pk + 1];
            if (e - b > kSmallBucket) {
                ws.big[1 + atomicAdd(&ws.big[0], 1)] = (int)pk;
                continue;
            }
            for (int i = b + 1; i < e; ++i) {
                const int v = ws.ids[i];
                int jx = i - 1;
                while (jx >= b && ws.ids[jx] > v) {
                    ws.ids[jx + 1] = ws.ids[jx];
                    --jx;
                }
                ws.ids[jx + 1] = v;
            }
        }
        if (sync()) return;
        // the large buckets: one block each, merge sort with all threads (runs of width w
        // merged pairwise per pass, output element k of a pair found by a merge-path binary
        // search; ids within a bucket are distinct).  Scratch: the bucket's range of `key`
        // (dead after the fill).  O(n log^2 n / threads) per bucket.
        const int nbig = ws.big[0];
        for (int i = bid; i < nbig; i += nblk) {
            const int pk = ws.big[1 + i];
            const int b = ws.offs[pk], n = ws.offs[pk + 1] - b;
            int* src = ws.ids + b;
            int* dst = ws.key + b;
            for (int w = 1; w < n; w <<= 1) {
                for (int k0 = tid; k0 < n; k0 += 256) {
                    const int s0 = (k0 / (2 * w)) * (2 * w);
                    const int mm = min(s0 + w, n), e = min(s0 + 2 * w, n);
                    const int k = k0 - s0;
                    const int* A = src + s0;
                    const int* Bv = src + mm;
                    const int la = mm - s0, lb = e - mm;
                    int lo = max(0, k - lb), hi = min(k, la);
                    while (lo < hi) {  // number of A's elements among the pair's first k outputs
                        const int mid = (lo + hi) >> 1;
                        if (A[mid] < Bv[k - 1 - mid])
                            lo = mid + 1;
                        else
                            hi = mid;
                    }
                    const int ib = k - lo;
                    dst[k0] = (lo < la && (ib >= lb || A[lo] < Bv[ib])) ? A[lo] : Bv[ib];
                }
                __syncthreads();
                int* t = src;
                src = dst;
                dst = t;
            }
            if (src != ws.ids + b)
                for (int k0 = tid; k0 < n; k0 += 256) ws.ids[b + k0] = src[k0];
            __syncthreads();
        }
        if (sync()) return;
        // texel t of plane pc0 + pl: its four nw-tap buckets (the samples having it as nw,
        // ne, sw, se tap) merged by the reference's order key; fractions from the position
        for (int64_t q = gtid; q < nq; q += gstride) {
            const int pl = (int)(q / HW);
            const int t = (int)(q - pl * HW);
            const int ty = t / g.W, tx = t - ty * g.W;
            const float* h = homs + (int64_t)(pc0 + pl) * 9;
            const int64_t base = pl * K;
            const int64_t bk[4] = {base + (int64_t)(ty + 1) * K1 + tx + 1, base + (int64_t)(ty + 1) * K1 + tx,
                                   base + (int64_t)ty * K1 + tx + 1, base + (int64_t)ty * K1 + tx};
            int pos[4], end[4];
            unsigned head[4];
#pragma unroll
            for (int c = 0; c < 4; ++c) {
                pos[c] = ws.offs[bk[c]];
                end[c] = ws.offs[bk[c] + 1];
                head[c] = pos[c] < end[c] ? order_key(ws.ids[pos[c]], c) : 0xFFFFFFFFu;
            }
            const float4* dsp = ds_plane(ws, pc0 + pl, HW);
            float a0 = 0.0f, a1 = 0.0f, a2 = 0.0f, a3 = 0.0f;
            for (;;) {
                int c = 0;
                unsigned m = head[0];
#pragma unroll
                for (int k = 1; k < 4; ++k)
                    if (head[k] < m) {
                        m = head[k];
                        c = k;
                    }
                if (m == 0xFFFFFFFFu) break;
                int pix = 0;
#pragma unroll
                for (int k = 0; k < 4; ++k) {  // static indexing keeps pos/head in registers
                    if (k == c) {
                        pix = ws.ids[pos[k]];
                        ++pos[k];
                        head[k] = pos[k] < end[k] ? order_key(ws.ids[pos[k]], k) : 0xFFFFFFFFu;
                    }
                }
                const int py_ = pix / g.W;
                float px, py;
                render_pos<FAST>(h, (float)(pix - py_ * g.W), (float)py_, g, px, py);
                const float wx = px - floorf(px), ex = 1.0f - wx;
                const float wy = py - floorf(py), sy = 1.0f - wy;
                const float w = ((c & 2) ? wy : sy) * ((c & 1) ? wx : ex);
                const float4 d = dsp[pix];
                a0 = a0 + w * d.x;
                a1 = a1 + w * d.y;
                a2 = a2 + w * d.z;
                a3 = a3 + w * d.w;
            }
            dmpi[(int64_t)t * g.P + pc0 + pl] = make_float4(a0, a1, a2, a3);
        }
        if (sync()) return;  // the chunk's arrays are reused by the next one
    }
}
#endif

// The ticket schedule's two steps, written for wave 0 of a block with WAVE-UNIFORM control flow
// (all 64 lanes run the wait loop and leave it together).  A first version ran them under
// `if (threadIdx.x == 0)` at the top of the item loop; the compiler's structurizer then split
// that lane's path from its wave's other lanes, which went round the barriers on their own
// (scalar s_barrier instructions run whatever the exec mask) and read a stale ticket: every
// box run hung, even a single block with trivial items (round 4, tools/ticket_selftest.py).
// Returns the block's next item (ticket) or -1 (none left, or aborted).
// A wait gives up after poll_limit polls (an A/B / test knob; ~0u in production) or after
// tick_limit wall-clock ticks (production: 60 s at the device's constant wall-clock rate; 0 = no
// time limit).  Giving up is never expected (the ticket argument above); a slow but correct wait --
// one block merge-sorting a huge bucket of a strongly minifying view -- takes seconds, not a minute.
__device__ __forceinline__ int fallback_ticket(unsigned* ticket, unsigned* done, int* abort_, int* aborted,
                                               unsigned total, unsigned nvirt, unsigned poll_limit,
                                               unsigned long long tick_limit, unsigned* timeouts,
                                               unsigned* next_fixed = nullptr) {
    const int lane = threadIdx.x & (kWave - 1);
    if (abort_ && __builtin_amdgcn_readfirstlane(
                      (int)__hip_atomic_load(abort_, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) != 0)
        return -1;
    unsigned tk = 0;
    if (next_fixed) {
        tk = *next_fixed;
        *next_fixed += nvirt;
    } else {
        if (lane == 0) tk = atomicAdd(ticket, 1u);
        tk = (unsigned)__builtin_amdgcn_readfirstlane((int)tk);
    }
    if (tk >= total) return -1;
    const unsigned need = tk / nvirt * nvirt;  // every item of the phases before this one done
    if (poll_limit == 0 && need > 0 && abort_) {  // tests: abort at the first wait
        if (lane == 0 && atomicExch(abort_, 1) == 0 && aborted) atomicAdd(aborted, 1);
        return -1;
    }
    const long long t0 = tick_limit ? wall_clock64() : 0;
    for (unsigned spins = 0;; ++spins) {
        const unsigned d = (unsigned)__builtin_amdgcn_readfirstlane(
            (int)__hip_atomic_load(done, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
        if (d >= need) break;
        if (abort_ && __builtin_amdgcn_readfirstlane(
                          (int)__hip_atomic_load(abort_, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) != 0)
            return -1;
        int give_up = spins > poll_limit;
        if (tick_limit && (spins & 63) == 63)
            give_up |= (unsigned long long)(wall_clock64() - t0) > tick_limit;
        if (__builtin_amdgcn_readfirstlane(give_up)) {
            if (lane == 0) {
                if (abort_ && atomicExch(abort_, 1) == 0 && aborted) atomicAdd(aborted, 1);
                if (timeouts) atomicAdd(timeouts, 1u);
            }
            return -1;
        }
        __builtin_amdgcn_s_sleep(2);
    }
    __threadfence();  // acquire: the earlier phases' stores are visible
    return (int)tk;
}

// after an item: every thread's stores, then one completion
__device__ __forceinline__ void fallback_done(unsigned* done) {
    __syncthreads();
    if (threadIdx.x == 0) {
        __threadfence();  // release: this item's stores before its completion
        atomicAdd(done, 1u);
    }
}

// One item of the fallback pipeline: virtual block bid (of nblk) of phase ph (0: zero the
// bucket sizes; 1 + kFbPhases * c + k: step k for plane chunk c)
template <bool FAST>
__device__ void bwd_fallback_item(const RenderGeom& g, const float* __restrict__ homs, const BwdWs& ws,
                                  float4* __restrict__ dmpi, int ph, int bid, int nblk, int* s_tmp, int p_lo,
                                  int p_hi) {
    const int tid = threadIdx.x;
    const int64_t gtid = (int64_t)bid * 256 + tid, gstride = (int64_t)nblk * 256;
    const int64_t HW = (int64_t)g.H * g.W;
    const int K1 = g.W + 1;
    const int64_t K = (int64_t)(g.H + 1) * K1;
    if (ph == 0) {  // bucket sizes start at zero (the fill returns them to zero for the next chunk)
        for (int64_t i = gtid; i < (int64_t)ws.pc * K; i += gstride) ws.count[i] = 0;
        return;
    }
    const int pc0 = p_lo + (ph - 1) / kFbPhases * ws.pc;
    const int step = (ph - 1) % kFbPhases;
    const int pcn = min(ws.pc, p_hi - pc0);
    const int64_t nq = pcn * HW, nk = pcn * K;
    const int nb = (int)((nk + kScanTile - 1) / kScanTile);
    switch (step) {
        case 0:  // nw-tap bucket of every (plane of the chunk, pixel) sample; sizes counted
            for (int64_t q = gtid; q < nq; q += gstride) {
                const int pl = (int)(q / HW);
                const int pix = (int)(q - pl * HW);
                const int y = pix / g.W, x = pix - y * g.W;
                float px, py;
                render_pos<FAST>(homs + (int64_t)(pc0 + pl) * 9, (float)x, (float)y, g, px, py);
                const float fx0 = floorf(px), fy0 = floorf(py);
                // some tap lies in the image iff the nw tap is in [-1, W-1] x [-1, H-1] (NaN: none)
                const bool in = fx0 >= -1.0f && fx0 <= (float)(g.W - 1) && fy0 >= -1.0f && fy0 <= (float)(g.H - 1);
                const int k = in ? ((int)fy0 + 1) * K1 + (int)fx0 + 1 : -1;
                ws.key[q] = k;
                if (in) atomicAdd(&ws.count[pl * K + k], 1);
            }
            return;
        case 1:  // exclusive scan of the sizes: tile sums
            for (int tb = bid; tb < nb; tb += nblk) {
                const int64_t base = (int64_t)tb * kScanTile + (int64_t)tid * kScanItems;
                int sum = 0;
                for (int i = 0; i < kScanItems; ++i)
                    if (base + i < nk) sum += ws.count[base + i];
                int total;
                block_exclusive_scan(sum, s_tmp, total);
                if (tid == 0) ws.bsum[tb] = total;
            }
            return;
        case 2:  // their scan (one block)
            if (bid == 0) {
                int carry = 0;
                for (int c0 = 0; c0 < nb; c0 += kScanBlock) {
                    const int i = c0 + tid;
                    const int v = i < nb ? ws.bsum[i] : 0;
                    int total;
                    const int ex = block_exclusive_scan(v, s_tmp, total);
                    if (i < nb) ws.bsum[i] = carry + ex;
                    carry += total;
                }
                if (tid == 0) ws.big[0] = 0;
            }
            return;
        case 3:  // per-tile apply
            for (int tb = bid; tb < nb; tb += nblk) {
                const int64_t base = (int64_t)tb * kScanTile + (int64_t)tid * kScanItems;
                int v[kScanItems];
                int sum = 0;
#pragma unroll
                for (int i = 0; i < kScanItems; ++i) {
                    v[i] = base + i < nk ? ws.count[base + i] : 0;
                    sum += v[i];
                }
                int total;
                int run = ws.bsum[tb] + block_exclusive_scan(sum, s_tmp, total);
#pragma unroll
                for (int i = 0; i < kScanItems; ++i) {
                    if (base + i < nk) ws.offs[base + i] = run;
                    run += v[i];
                }
                if (tb == nb - 1 && tid == kScanBlock - 1) ws.offs[nk] = run;  // grand total
            }
            return;
        case 4:  // pixel ids into their buckets (atomic slot claim; sizes return to zero)
            for (int64_t q = gtid; q < nq; q += gstride) {
                const int k = ws.key[q];
                if (k < 0) continue;
                const int64_t pl = q / HW;
                const int64_t pk = pl * K + k;
                const int slot = atomicSub(&ws.count[pk], 1) - 1;
                ws.ids[ws.offs[pk] + slot] = (int)(q - pl * HW);
            }
            return;
        case 5:  // each bucket sorted by pixel id: <= kSmallBucket ids by one thread (insertion
                 // sort), larger ones (minification, degenerate homographies) listed for a block
            for (int64_t pk = gtid; pk < nk; pk += gstride) {
                const int b = ws.offs[pk], e = ws.offs[pk + 1];
                if (e - b > kSmallBucket) {
                    ws.big[1 + atomicAdd(&ws.big[0], 1)] = (int)pk;
                    continue;
                }
                for (int i = b + 1; i < e; ++i) {
                    const int v = ws.ids[i];
                    int jx = i - 1;
                    while (jx >= b && ws.ids[jx] > v) {
                        ws.ids[jx + 1] = ws.ids[jx];
                        --jx;
                    }
                    ws.ids[jx + 1] = v;
                }
            }
            return;
        case 6: {  // the large buckets: one block each, merge sort with all threads (runs of width
                   // w merged pairwise per pass, output element k of a pair found by a merge-path
                   // binary search; ids within a bucket are distinct).  Scratch: the bucket's range
                   // of `key` (dead after the fill).  O(n log^2 n / threads) per bucket.
            const int nbig = ws.big[0];
            for (int i = bid; i < nbig; i += nblk) {
                const int pk = ws.big[1 + i];
                const int b = ws.offs[pk], n = ws.offs[pk + 1] - b;
                int* src = ws.ids + b;
                int* dst = ws.key + b;
                for (int w = 1; w < n; w <<= 1) {
                    for (int k0 = tid; k0 < n; k0 += 256) {
                        const int s0 = (k0 / (2 * w)) * (2 * w);
                        const int mm = min(s0 + w, n), e = min(s0 + 2 * w, n);
                        const int k = k0 - s0;
                        const int* A = src + s0;
                        const int* Bv = src + mm;
                        const int la = mm - s0, lb = e - mm;
                        int lo = max(0, k - lb), hi = min(k, la);
                        while (lo < hi) {  // number of A's elements among the pair's first k outputs
                            const int mid = (lo + hi) >> 1;
                            if (A[mid] < Bv[k - 1 - mid])
                                lo = mid + 1;
                            else
                                hi = mid;
                        }
                        const int ib = k - lo;
                        dst[k0] = (lo < la && (ib >= lb || A[lo] < Bv[ib])) ? A[lo] : Bv[ib];
                    }
                    __syncthreads();
                    int* t = src;
                    src = dst;
                    dst = t;
                }
                if (src != ws.ids + b)
                    for (int k0 = tid; k0 < n; k0 += 256) ws.ids[b + k0] = src[k0];
                __syncthreads();
            }
            return;
        }
        default:  // texel t of plane pc0 + pl: its four nw-tap buckets (the samples having it as nw,
                  // ne, sw, se tap) merged by the reference's order key; fractions from the position
            for (int64_t q = gtid; q < nq; q += gstride) {
                const int pl = (int)(q / HW);
                const int t = (int)(q - pl * HW);
                const int ty = t / g.W, tx = t - ty * g.W;
                const float* h = homs + (int64_t)(pc0 + pl) * 9;
                const int64_t base = pl * K;
                const int64_t bk[4] = {base + (int64_t)(ty + 1) * K1 + tx + 1, base + (int64_t)(ty + 1) * K1 + tx,
                                       base + (int64_t)ty * K1 + tx + 1, base + (int64_t)ty * K1 + tx};
                int pos[4], end[4];
                unsigned head[4];
#pragma unroll
                for (int c = 0; c < 4; ++c) {
                    pos[c] = ws.offs[bk[c]];
                    end[c] = ws.offs[bk[c] + 1];
                    head[c] = pos[c] < end[c] ? order_key(ws.ids[pos[c]], c) : 0xFFFFFFFFu;
                }
                const float4* dsp = ds_plane(ws, pc0 + pl, HW);
                float a0 = 0.0f, a1 = 0.0f, a2 = 0.0f, a3 = 0.0f;
                for (;;) {
                    int c = 0;
                    unsigned m = head[0];
#pragma unroll
                    for (int k = 1; k < 4; ++k)
                        if (head[k] < m) {
                            m = head[k];
                            c = k;
                        }
                    if (m == 0xFFFFFFFFu) break;
                    int pix = 0;
#pragma unroll
                    for (int k = 0; k < 4; ++k) {  // static indexing keeps pos/head in registers
                        if (k == c) {
                            pix = ws.ids[pos[k]];
                            ++pos[k];
                            head[k] = pos[k] < end[k] ? order_key(ws.ids[pos[k]], k) : 0xFFFFFFFFu;
                        }
                    }
                    const int py_ = pix / g.W;
                    float px, py;
                    render_pos<FAST>(h, (float)(pix - py_ * g.W), (float)py_, g, px, py);
                    const float wx = px - floorf(px), ex = 1.0f - wx;
                    const float wy = py - floorf(py), sy = 1.0f - wy;
                    const float w = ((c & 2) ? wy : sy) * ((c & 1) ? wx : ex);
                    const float4 d = dsp[pix];
                    a0 = a0 + w * d.x;
                    a1 = a1 + w * d.y;
                    a2 = a2 + w * d.z;
                    a3 = a3 + w * d.w;
                }
                dmpi[(int64_t)t * g.P + pc0 + pl] = make_float4(a0, a1, a2, a3);
            }
            return;
    }
}

// flag words: [0] run the fallback, [1] next ticket, [2] items done, [3] this view aborted,
// [4] views aborted in this call (sticky; zeroed by mpiv_render_backward's first memset)
template <bool FAST>
// fixed != 0 (A/B diagnosis): block b takes items b, b + nblk, ... in order instead of tickets
// (the grid-barrier schedule: needs every block resident)
// planes [p_lo, p_hi) (a plane group of mpiv_render_backward, or all of them)
// poison_n > 0 (round 6, the single-group schedule): bwd_poison_kernel's NaN fill of an aborted
// view (its poison_n d MPI texels) by the last block to leave, instead of a launch of its own after
// every view.
__global__ __launch_bounds__(256) void bwd_fallback_kernel(RenderGeom g, const float* __restrict__ homs,
                                                                  BwdWs ws, float4* __restrict__ dmpi,
                                                                  unsigned poll_limit, unsigned long long tick_limit,
                                                                  int fixed, int p_lo, int p_hi, int64_t poison_n = 0) {
    __shared__ int s_tmp[kScanBlock];
    __shared__ int s_ticket;
    if (ws.flag[0] == 0) return;  // uniform over the grid: the tile gather was complete
    const int nblk = gridDim.x, tid = threadIdx.x;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // scalar: wave-uniform branches only
    const int nchunk = (p_hi - p_lo + ws.pc - 1) / ws.pc;
    const unsigned total = (unsigned)(1 + kFbPhases * nchunk) * (unsigned)nblk;
    unsigned* ticket = reinterpret_cast<unsigned*>(ws.flag + 1);
    unsigned* done = reinterpret_cast<unsigned*>(ws.flag + 2);
    unsigned next_fixed = blockIdx.x;
    for (;;) {
        if (wave == 0) {
            const int t = fallback_ticket(ticket, done, ws.flag + 3, ws.vcount, total, (unsigned)nblk, poll_limit,
                                          tick_limit, nullptr, fixed ? &next_fixed : nullptr);
            if (tid == 0) s_ticket = t;
        }
        __syncthreads();
        const int t = __builtin_amdgcn_readfirstlane(s_ticket);
        __syncthreads();  // s_ticket is rewritten by the next iteration
        if (t < 0) {
            if (poison_n > 0 && last_block_in(ws.flag + kFlagFallbackExit, &s_ticket) &&
                __hip_atomic_load(ws.flag + 3, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0) {
                const float q = __builtin_nanf("");
                if (tid == 0 && ws.sink) __hip_atomic_store(ws.sink, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                for (int64_t i = tid; i < poison_n; i += 256) dmpi[i] = make_float4(q, q, q, q);
            }
            return;
        }
        bwd_fallback_item<FAST>(g, homs, ws, dmpi, t / nblk, t % nblk, nblk, s_tmp, p_lo, p_hi);
        fallback_done(done);
    }
}




#if MPIV_AB
// Ticket-protocol self-test (diagnosis of bwd_fallback_ticket_kernel): the same ticket / wait /
// completion code with trivial items -- item (phase q, virtual block b) checks that every item
// of phase q-1 has left its mark, counts the ones missing in ctr[2], and marks marks[q][b].
// ctr: [0] tickets, [1] completions, [2] violations, [3] aborted waits (zeroed by the caller).
__global__ __launch_bounds__(256) void ticket_selftest_kernel(unsigned* __restrict__ ctr, int* __restrict__ marks,
                                                              int nphase, int nvirt, unsigned poll_limit) {
    const int tid = threadIdx.x;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // scalar: wave-uniform branches only
    const unsigned total = (unsigned)nphase * (unsigned)nvirt;
    __shared__ int s_ticket;
    for (;;) {
        if (wave == 0) {
            const int t = fallback_ticket(ctr, ctr + 1, nullptr, nullptr, total, (unsigned)nvirt, poll_limit, 0ull,
                                          ctr + 3);
            if (tid == 0) s_ticket = t;
        }
        __syncthreads();
        const int t = __builtin_amdgcn_readfirstlane(s_ticket);
        __syncthreads();
        if (t < 0) return;
        const int q = t / nvirt, b = t % nvirt;
        unsigned bad = 0;
        if (q > 0)
            for (int i = tid; i < nvirt; i += 256) bad += marks[(q - 1) * nvirt + i] != 1;
        if (bad) atomicAdd(ctr + 2, bad);
        if (tid == 0) marks[q * nvirt + b] = 1;
        fallback_done(ctr + 1);
    }
}
#endif

// After the fallback: a view whose pipeline aborted (flag[3], or flag_b[3] of the overlapped
// schedule's second counter set) gets a NaN gradient; count (non-null: the overlapped schedule,
// whose fallbacks do not count) adds the view once
__global__ __launch_bounds__(256) void bwd_poison_kernel(const int* __restrict__ flag, float4* __restrict__ dmpi,
                                                         int64_t n, const int* __restrict__ flag_b = nullptr,
                                                         int* __restrict__ count = nullptr, int* sink = nullptr) {
    if (flag[3] == 0 && (!flag_b || flag_b[3] == 0)) return;
    if (count && blockIdx.x == 0 && threadIdx.x == 0) atomicAdd(count, 1);
    if (sink && blockIdx.x == 0 && threadIdx.x == 0) __hip_atomic_store(sink, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    const float q = __builtin_nanf("");
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256)
        dmpi[i] = make_float4(q, q, q, q);
}

}  // namespace mpiv
