// render_bwd.hip -- d(render)/d(MPI): the adjoint of the fused warp + over-composite
// (autograd of mpi_render_view_torch, utils.py:267-294, w.r.t. rgba_layers), BIT-EXACT
// to the reference's autograd on CPU (oracle/mpiv_oracle.c oracle_render_backward,
// pinned to tests/golden/grad.npz).
//
// The reference's gradient is a float sum per source texel whose ORDER is fixed by
// ATen's grid_sampler_2d_backward CPU kernel: per (plane, view) slice the output
// pixels are walked in flat chunks of 8; per chunk and channel the corners nw, ne,
// sw, se are scattered over the chunk's lanes in order.  A GPU scatter with float
// atomics would add in arrival order (nondeterministic, not bit-exact), so the
// adjoint is computed as a deterministic GATHER instead:
//
//  1. chain  (one work-item per output pixel, planes back to front then front to
//            back): recompute the forward (same recipe as render.hip), keep the
//            prefix out_{p-1} and the sample s_p per plane in the workspace, then
//            walk the over-chain backwards exactly like autograd's Mul/Rsub
//            backward: d rgb = g*a, d a = sum(g*rgb) + -(sum(g*out_{p-1})),
//            g *= (1 - a).  Each (plane, pixel) also records its bilinear fractions
//            and the bucket of its north-west tap; bucket sizes are counted.
//  2. scan   exclusive prefix sum of the bucket sizes (3 kernels).
//  3. bucket pixel ids into their buckets (atomic slot claim), then sort each
//            bucket by pixel id: buckets of <= kSmallBucket ids (~1 pixel for
//            non-minifying warps) by one thread, larger ones (minification, degenerate
//            homographies: up to every pixel of a plane in one bucket) by a block-wide
//            merge sort, so no bucket size costs O(n^2) on one lane.
//  4. gather (one work-item per source texel): the texel is the nw tap of bucket
//            (x, y), the ne tap of bucket (x-1, y), sw of (x, y-1), se of (x-1, y-1);
//            the four sorted lists are merged by the reference's order key
//            (pixel/8, corner, pixel%8) and summed in that order, from +0.
// Every product and sum is a single fp32 rounding written out explicitly (the
// library builds with -ffp-contract=off).
#include "mpiv_common.hpp"

namespace mpiv {

constexpr int kGridVec = 8;       // grid_sampler_2d_backward chunk width (oracle.GRID_VEC)
constexpr int kScanItems = 16;    // items per thread in the bucket scan
constexpr int kScanBlock = 256;
constexpr int kScanTile = kScanItems * kScanBlock;

constexpr int kSmallBucket = 32;  // larger buckets are sorted by a whole block

struct BwdWs {
    float4* prev;  // [P][HW]  out_{p-1} (rgb, 0)
    float4* ds;    // [P][HW]  sample s_p, then d s_p = (d rgb, d a)
    float2* fw;    // [P][HW]  bilinear fractions (wx, wy)
    int* key;      // [P][HW]  nw-tap bucket in the (H+1) x (W+1) grid, -1 = no tap in the image;
                   //          after the fill: merge-sort scratch (same offsets as ids)
    int* count;    // [P*K]    bucket sizes; zero on entry and on exit of every view
    int* offs;     // [P*K+1]  exclusive scan of count
    int* ids;      // [P*HW]   pixel ids grouped by bucket
    int* bsum;     // scan block sums
    int* big;      // [0] = number of large buckets, [1..] their indices (P*HW/(kSmallBucket+1) max)
};

// ---- 1. forward recompute + over-chain adjoint, one work-item per output pixel ----
template <bool FAST>
__global__ __launch_bounds__(256) void render_bwd_chain_kernel(const float4* __restrict__ planes,
                                                               int64_t plane_stride, RenderGeom g,
                                                               const float* __restrict__ homs,
                                                               const float* __restrict__ dout, BwdWs ws) {
    const int tiles_x = (g.W + kTileX - 1) / kTileX;
    const int x = (blockIdx.x % tiles_x) * kTileX + (threadIdx.x & (kWave - 1));
    const int y = (blockIdx.x / tiles_x) * kTileY + (threadIdx.x >> 6);
    if (x >= g.W || y >= g.H) return;
    const int HW = g.H * g.W;
    const int pix = y * g.W + x;
    const int K1 = g.W + 1;
    const int K = (g.H + 1) * K1;
    const float fx = (float)x, fy = (float)y;

    float cr = -0.0f, cg = -0.0f, cb = -0.0f;  // plane 0 replaces it exactly (render.hip)
    // plane p's sample: position, then its four taps in flight (the last plane is
    // re-issued past the end so every iteration issues; render.hip's ping-pong)
    struct Sample {
        TapSet ts;
        float px, py;
    };
    auto issue = [&](int p, Sample& sm) {
        const int pc = p < g.P ? p : g.P - 1;
        render_pos<FAST>(homs + (int64_t)pc * 9, fx, fy, g, sm.px, sm.py);
        issue_taps_padded(make_rsrc(planes + (int64_t)pc * plane_stride, g.plane_bytes), g.W, g.H, g.Wp, g.org,
                          g.row, sm.px, sm.py, sm.ts);
    };
    auto consume = [&](int p, const Sample& sm) {
        const f32x4 s = blend_taps(sm.ts);
        const float fx0 = floorf(sm.px), fy0 = floorf(sm.py);
        const int64_t q = (int64_t)p * HW + pix;
        ws.fw[q] = make_float2(sm.px - fx0, sm.py - fy0);
        // some tap of this sample lies in the image iff the nw tap is in [-1, W-1] x [-1, H-1]
        // (float compares: NaN positions have no taps, as in the reference's masks)
        const bool in = fx0 >= -1.0f && fx0 <= (float)(g.W - 1) && fy0 >= -1.0f && fy0 <= (float)(g.H - 1);
        const int k = in ? ((int)fy0 + 1) * K1 + (int)fx0 + 1 : -1;
        ws.key[q] = k;
        if (in) atomicAdd(&ws.count[(int64_t)p * K + k], 1);
        ws.prev[q] = make_float4(cr, cg, cb, 0.0f);
        ws.ds[q] = make_float4(s[0], s[1], s[2], s[3]);
        const float a = p == 0 ? 1.0f : s[3];
        const float om = 1.0f - a;
        cr = over(s[0], a, om, cr);
        cg = over(s[1], a, om, cg);
        cb = over(s[2], a, om, cb);
    };
    Sample A, B;
    issue(0, A);
    int p = 0;
    for (; p + 1 < g.P; p += 2) {
        issue(p + 1, B);
        __builtin_amdgcn_sched_barrier(0);
        consume(p, A);
        issue(p + 2, A);
        __builtin_amdgcn_sched_barrier(0);
        consume(p + 1, B);
    }
    if (p < g.P) consume(p, A);
    // over_composite backward (utils.py:149-156 under autograd), front to back
    const float* d = dout + (int64_t)pix * 3;
    float g0 = d[0], g1 = d[1], g2 = d[2];
    for (int p = g.P - 1; p >= 1; --p) {
        const int64_t q = (int64_t)p * HW + pix;
        const float4 s = ws.ds[q];
        const float4 o = ws.prev[q];
        const float a = s.w, om = 1.0f - a;
        float s1 = g0 * s.x;
        s1 = s1 + g1 * s.y;
        s1 = s1 + g2 * s.z;
        float s2 = g0 * o.x;
        s2 = s2 + g1 * o.y;
        s2 = s2 + g2 * o.z;
        ws.ds[q] = make_float4(g0 * a, g1 * a, g2 * a, s1 + (-s2));
        g0 = g0 * om;
        g1 = g1 * om;
        g2 = g2 * om;
    }
    ws.ds[pix] = make_float4(g0, g1, g2, 0.0f);  // plane 0: output = rgb_0, alpha unused
}

// ---- 2. exclusive scan of the bucket sizes -------------------------------------------

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

__global__ __launch_bounds__(kScanBlock) void scan_tile_sums_kernel(const int* __restrict__ in, int64_t n,
                                                                    int* __restrict__ bsum) {
    __shared__ int s_tmp[kScanBlock];
    const int64_t base = (int64_t)blockIdx.x * kScanTile + (int64_t)threadIdx.x * kScanItems;
    int sum = 0;
    if (base + kScanItems <= n) {  // whole item run in range: 16-B loads (base is 64-B aligned)
        const int4* v4 = reinterpret_cast<const int4*>(in + base);
#pragma unroll
        for (int i = 0; i < kScanItems / 4; ++i) {
            const int4 v = v4[i];
            sum += v.x + v.y + v.z + v.w;
        }
    } else {
#pragma unroll
        for (int i = 0; i < kScanItems; ++i)
            if (base + i < n) sum += in[base + i];
    }
    int total;
    block_exclusive_scan(sum, s_tmp, total);
    if (threadIdx.x == 0) bsum[blockIdx.x] = total;
}

// single block: exclusive scan of the nb tile sums in place
__global__ __launch_bounds__(kScanBlock) void scan_tile_offsets_kernel(int* __restrict__ bsum, int nb) {
    __shared__ int s_tmp[kScanBlock];
    int carry = 0;
    for (int c0 = 0; c0 < nb; c0 += kScanBlock) {
        const int i = c0 + threadIdx.x;
        const int v = i < nb ? bsum[i] : 0;
        int total;
        const int ex = block_exclusive_scan(v, s_tmp, total);
        if (i < nb) bsum[i] = carry + ex;
        carry += total;
    }
}

__global__ __launch_bounds__(kScanBlock) void scan_apply_kernel(const int* __restrict__ in, int64_t n,
                                                                const int* __restrict__ bsum,
                                                                int* __restrict__ out) {
    __shared__ int s_tmp[kScanBlock];
    const int64_t base = (int64_t)blockIdx.x * kScanTile + (int64_t)threadIdx.x * kScanItems;
    int v[kScanItems];
    int sum = 0;
    const bool full = base + kScanItems <= n;  // whole run in range: 16-B loads and stores
    if (full) {
        const int4* v4 = reinterpret_cast<const int4*>(in + base);
#pragma unroll
        for (int i = 0; i < kScanItems / 4; ++i) {
            const int4 q = v4[i];
            v[4 * i] = q.x; v[4 * i + 1] = q.y; v[4 * i + 2] = q.z; v[4 * i + 3] = q.w;
        }
    } else {
#pragma unroll
        for (int i = 0; i < kScanItems; ++i) v[i] = base + i < n ? in[base + i] : 0;
    }
#pragma unroll
    for (int i = 0; i < kScanItems; ++i) sum += v[i];
    int total;
    int run = bsum[blockIdx.x] + block_exclusive_scan(sum, s_tmp, total);
    if (full) {  // out = offs + 0: 16-B aligned like in
        int4* o4 = reinterpret_cast<int4*>(out + base);
#pragma unroll
        for (int i = 0; i < kScanItems / 4; ++i) {
            int4 q;
            q.x = run; run += v[4 * i];
            q.y = run; run += v[4 * i + 1];
            q.z = run; run += v[4 * i + 2];
            q.w = run; run += v[4 * i + 3];
            o4[i] = q;
        }
    } else {
#pragma unroll
        for (int i = 0; i < kScanItems; ++i) {
            if (base + i < n) out[base + i] = run;
            run += v[i];
        }
    }
    if (blockIdx.x == gridDim.x - 1 && threadIdx.x == kScanBlock - 1) out[n] = run;  // grand total
}

// ---- 3. pixel ids into buckets, then each bucket sorted by pixel id ------------------

__global__ __launch_bounds__(256) void bucket_fill_kernel(int P, int HW, int K, BwdWs ws) {
    const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= (int64_t)P * HW) return;
    const int k = ws.key[q];
    if (k < 0) return;
    const int p = (int)(q / HW), pix = (int)(q - (int64_t)p * HW);
    const int64_t pk = (int64_t)p * K + k;
    const int slot = atomicSub(&ws.count[pk], 1) - 1;  // count returns to 0 for the next view
    ws.ids[ws.offs[pk] + slot] = pix;
}

__global__ __launch_bounds__(256) void bucket_sort_kernel(int64_t nbuckets, BwdWs ws) {
    const int64_t pk = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (pk >= nbuckets) return;
    const int b = ws.offs[pk], e = ws.offs[pk + 1];
    if (e - b > kSmallBucket) {  // left to big_bucket_sort_kernel
        ws.big[1 + atomicAdd(&ws.big[0], 1)] = (int)pk;
        return;
    }
    for (int i = b + 1; i < e; ++i) {  // insertion sort (at most kSmallBucket ids)
        const int v = ws.ids[i];
        int j = i - 1;
        while (j >= b && ws.ids[j] > v) {
            ws.ids[j + 1] = ws.ids[j];
            --j;
        }
        ws.ids[j + 1] = v;
    }
}

// Sorts the large buckets listed by bucket_sort_kernel: each block takes buckets
// blockIdx.x, blockIdx.x + gridDim.x, ... and merge-sorts one at a time, all threads
// together (runs of width w merged pairwise per pass; output element k of a pair found
// by a merge-path binary search; ids within a bucket are distinct).  The scratch is the
// bucket's range of `key` (dead after the fill).  O(n log^2 n / threads) per bucket.
__global__ __launch_bounds__(256) void big_bucket_sort_kernel(BwdWs ws) {
    const int nbig = ws.big[0];
    for (int i = blockIdx.x; i < nbig; i += gridDim.x) {
        const int pk = ws.big[1 + i];
        const int b = ws.offs[pk], n = ws.offs[pk + 1] - b;
        int* src = ws.ids + b;
        int* dst = ws.key + b;
        for (int w = 1; w < n; w <<= 1) {
            for (int k0 = threadIdx.x; k0 < n; k0 += blockDim.x) {
                const int s0 = (k0 / (2 * w)) * (2 * w);
                const int m = min(s0 + w, n), e = min(s0 + 2 * w, n);
                const int k = k0 - s0;
                const int* A = src + s0;
                const int* Bv = src + m;
                const int la = m - s0, lb = e - m;
                int lo = max(0, k - lb), hi = min(k, la);
                while (lo < hi) {  // number of A's elements among the pair's first k outputs
                    const int mid = (lo + hi) >> 1;
                    if (A[mid] < Bv[k - 1 - mid]) lo = mid + 1;
                    else hi = mid;
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
            for (int k0 = threadIdx.x; k0 < n; k0 += blockDim.x) ws.ids[b + k0] = src[k0];
        __syncthreads();
    }
}

// ---- 4. per-texel gather in the reference's scatter order ----------------------------

struct GradOut {
    int64_t y, x, p, c;  // element strides of one view of d rgba_layers [H, W, P, 4]
};

__device__ __forceinline__ unsigned order_key(int pix, int corner) {
    return ((unsigned)(pix / kGridVec) << 5) | ((unsigned)corner << 3) | (unsigned)(pix % kGridVec);
}

// Sum of the gradient contributions of texel t of plane p, in the reference's order.
__device__ __forceinline__ float4 gather_texel(int H, int W, int p, int t, const BwdWs& ws) {
    const int HW = H * W;
    const int ty = t / W, tx = t - ty * W;
    const int K1 = W + 1;
    const int64_t base = (int64_t)p * (H + 1) * K1;
    // the texel is the nw / ne / sw / se tap of the samples in these nw-tap buckets
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
    const float4* dsp = ws.ds + (int64_t)p * HW;
    const float2* fwp = ws.fw + (int64_t)p * HW;
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
        const float2 f = fwp[pix];
        const float wx = f.x, ex = 1.0f - wx;
        const float wy = f.y, sy = 1.0f - wy;
        const float w = c == 0 ? sy * ex : c == 1 ? sy * wx : c == 2 ? wy * ex : wy * wx;
        const float4 d = dsp[pix];
        a0 = a0 + w * d.x;
        a1 = a1 + w * d.y;
        a2 = a2 + w * d.z;
        a3 = a3 + w * d.w;
    }
    return make_float4(a0, a1, a2, a3);
}

// Generic output strides: one work-item per (plane, texel), planes outermost.
__global__ __launch_bounds__(256) void render_bwd_gather_kernel(int H, int W, int P, BwdWs ws,
                                                                float* __restrict__ dmpi, GradOut so) {
    const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int HW = H * W;
    if (q >= (int64_t)P * HW) return;
    const int p = (int)(q / HW), t = (int)(q - (int64_t)p * HW);
    const int ty = t / W, tx = t - ty * W;
    const float4 a = gather_texel(H, W, p, t, ws);
    float* o = dmpi + ty * so.y + tx * so.x + p * so.p;
    o[0] = a.x;
    o[so.c] = a.y;
    o[2 * so.c] = a.z;
    o[3 * so.c] = a.w;
}

// Dense output ([H,W,P,4] contiguous, 16-B aligned): a block gathers 64 texels x 8
// planes (wave = plane: the workspace reads stay coalesced) and writes them through
// LDS as one 128-B run per texel (8 planes x 16 B) -- the direct form writes 4-B pieces
// at a P*16-B lane stride.
constexpr int kGatherPl = 8;
__global__ __launch_bounds__(kGatherPl * 64) void render_bwd_gather_dense_kernel(int H, int W, int P, BwdWs ws,
                                                                              float4* __restrict__ dmpi) {
    __shared__ float4 tile[kGatherPl][kWave + 1];
    const int HW = H * W;
    const int t0 = blockIdx.x * kWave, p0 = blockIdx.y * kGatherPl;
    const int lane = threadIdx.x & (kWave - 1), w = threadIdx.x >> 6;
    const int t = t0 + lane, p = p0 + w;
    if (t < HW && p < P) tile[w][lane] = gather_texel(H, W, p, t, ws);
    __syncthreads();
    const int i = threadIdx.x / kGatherPl, j = threadIdx.x % kGatherPl;  // texel, plane (plane fastest)
    if (t0 + i < HW && p0 + j < P) dmpi[(int64_t)(t0 + i) * P + p0 + j] = tile[j][i];
}

}  // namespace mpiv
