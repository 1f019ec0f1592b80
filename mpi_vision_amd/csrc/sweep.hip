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

// Source images as 16-B texels with a 2-texel zero border (the render's packed-plane
// convention, mpiv_common.hpp issue_taps_padded): [B][Hs+4][Ws+4] float4, channels >= C
// zero.  Border texels are written as zeros, so the sweep needs no per-tap range test.
__global__ __launch_bounds__(256) void pad_texels_kernel(const float* __restrict__ img, ImgStrides s, int Hs,
                                                         int Ws, int C, FastDiv fd_wp, float4* __restrict__ out) {
    const int Wp = Ws + 2 * kPad;
    const int64_t npix = (int64_t)(Hs + 2 * kPad) * Wp;
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int b = blockIdx.y;
    if (i >= npix) return;
    const int yp = (int)fast_div((unsigned)i, fd_wp);
    const int y = yp - kPad, x = (int)i - yp * Wp - kPad;
    float v[4] = {0.f, 0.f, 0.f, 0.f};
    if ((unsigned)y < (unsigned)Hs && (unsigned)x < (unsigned)Ws) {
        const float* t = img + b * s.b + y * s.y + x * s.x;
        for (int c = 0; c < C && c < 4; ++c) v[c] = t[c * s.c];
    }
    out[b * npix + i] = make_float4(v[0], v[1], v[2], v[3]);
}

// Plane sweep over padded 16-B texels (C <= 4).  One work-item = one target pixel x a
// group of kSweepDG consecutive depths (group fastest, so a wave writes one contiguous
// run of the volume): the camera ray and the index math are shared by the group, its
// 4 x kSweepDG tap loads are in flight together, u/den and v/den share one reciprocal
// (div2_rn), the two launch-constant divisions (x / Hs, y / Ws) use div_const, and
// the group's kSweepDG*C results leave as 16-B stores when the output rows are
// 16-B aligned (VEC).
constexpr int kSweepDG = 4;
constexpr int kSweepMaxLdsD = 1024;  // depths staged in LDS up to this many planes

struct PadGeom {
    int Wp, org, row, plane_bytes;  // padded source plane: pitch (texels), (0,0) offset, row bytes, size
};

// STORE 0: scalar stores; 1: 16-B stores per lane (VEC rows); 2: the block's contiguous
// output run staged through LDS and written as 16-B stores by consecutive lanes (bare,
// dense volume only: out_pstride == NG*kSweepDG*C).
template <int C, int STORE>
__global__ __launch_bounds__(256) void plane_sweep_group_kernel(const float4* __restrict__ img4, SweepParams sp,
                                                                PadGeom pg, float rc_hs, float rc_ws, FastDiv fd_g,
                                                                FastDiv fd_w, const float* __restrict__ ki,
                                                                const float* __restrict__ proj,
                                                                const float* __restrict__ depths,
                                                                float* __restrict__ out, int64_t out_bstride,
                                                                int out_pstride) {
    __shared__ float s_dep[kSweepMaxLdsD];
    __shared__ float4 s_out[STORE == 2 ? 256 * C : 1];
    const bool lds_dep = sp.D <= kSweepMaxLdsD;
    if (lds_dep)
        for (int i = threadIdx.x; i < sp.D; i += blockDim.x) s_dep[i] = depths[i];
    __syncthreads();
    const int NG = (sp.D + kSweepDG - 1) / kSweepDG;
    const unsigned per_view = (unsigned)sp.Ht * sp.Wt * NG;  // < 2^31, checked on the host
    const unsigned gid0 = blockIdx.x * blockDim.x + threadIdx.x;
    const unsigned gid = STORE == 2 ? min(gid0, per_view - 1) : gid0;  // whole block reaches the barrier
    if (gid0 >= per_view && STORE != 2) return;
    const int b = blockIdx.y;
    const float* k9 = ki + (int64_t)b * 9;
    const float* m = proj + (int64_t)b * 16;
    const __amdgpu_buffer_rsrc_t r = make_rsrc(img4 + (int64_t)b * pg.plane_bytes / 16, pg.plane_bytes);
    const unsigned pix = fast_div(gid, fd_g);
    const int dg = (int)(gid - pix * NG);
    const unsigned yy = fast_div(pix, fd_w);
    const float fy = (float)(int)yy, fx = (float)(int)(pix - yy * sp.Wt);
    float rx, ry, rz;
    ray(k9, fx, fy, rx, ry, rz);  // pixel2cam_torch, utils.py:370
    TapSet t[kSweepDG];
#pragma unroll
    for (int j = 0; j < kSweepDG; ++j) {
        const int d = min(dg * kSweepDG + j, sp.D - 1);  // a partial last group recomputes depth D-1
        const float dep = lds_dep ? s_dep[d] : depths[d];
        const float X = rx * dep, Y = ry * dep, Z = rz * dep;
        const float pu = __builtin_fmaf(m[2], Z, __builtin_fmaf(m[1], Y, m[0] * X)) + m[3];
        const float pv = __builtin_fmaf(m[6], Z, __builtin_fmaf(m[5], Y, m[4] * X)) + m[7];
        const float pz = __builtin_fmaf(m[10], Z, __builtin_fmaf(m[9], Y, m[8] * X)) + m[11];
        float su, sv;
        div2_rn(pu, pv, pz + 1e-10f, su, sv);  // cam2pixel_torch, utils.py:388-391
        const float cx = div_const(su + 0.5f, sp.fhs, rc_hs);  // SWAPPED: x / H, utils.py:444
        const float cy = div_const(sv + 0.5f, sp.fws, rc_ws);  //          y / W
        issue_taps_padded(r, sp.Ws, sp.Hs, pg.Wp, pg.org, pg.row, unnormalize(to_grid(cx), sp.half_ws),
                          unnormalize(to_grid(cy), sp.half_hs), t[j]);
    }
    float v[kSweepDG * C];
#pragma unroll
    for (int j = 0; j < kSweepDG; ++j) {
        const f32x4 s = blend_taps(t[j]);
#pragma unroll
        for (int c = 0; c < C; ++c) v[j * C + c] = s[c];
    }
    if (STORE == 2) {
        // dense volume: item g's kSweepDG*C floats sit at g*kSweepDG*C of this view
#pragma unroll
        for (int k = 0; k < C; ++k)
            s_out[threadIdx.x * C + k] = make_float4(v[4 * k], v[4 * k + 1], v[4 * k + 2], v[4 * k + 3]);
        __syncthreads();
        const unsigned n4 = per_view * C;  // float4s in this view's volume
        float4* ov = reinterpret_cast<float4*>(out + (int64_t)b * out_bstride);
        const unsigned blk0 = blockIdx.x * blockDim.x * C;
#pragma unroll
        for (int k = 0; k < C; ++k) {
            const unsigned i = k * blockDim.x + threadIdx.x;
            if (blk0 + i < n4) ov[blk0 + i] = s_out[i];
        }
        return;
    }
    float* o = out + (int64_t)b * out_bstride + (int64_t)pix * out_pstride + dg * kSweepDG * C;
    if (STORE == 1 && (dg + 1) * kSweepDG <= sp.D) {
#pragma unroll
        for (int k = 0; k < C; ++k)  // kSweepDG * C floats = C float4
            reinterpret_cast<float4*>(o)[k] = make_float4(v[4 * k], v[4 * k + 1], v[4 * k + 2], v[4 * k + 3]);
    } else {
        const int nd = min(kSweepDG, sp.D - dg * kSweepDG);
#pragma unroll
        for (int j = 0; j < kSweepDG; ++j)
            if (j < nd)
#pragma unroll
                for (int c = 0; c < C; ++c) o[j * C + c] = v[j * C + c];
    }
}

// Tile sweep: a block owns 64 consecutive target pixels (flat index) of one view and
// sweeps them through all depths; lane = pixel, so each tap load of a wave reads ~64
// consecutive source texels (one depth: near-constant disparity), the access shape
// the vector L1 serves fastest, instead of texels scattered along 16 epipolar
// segments.  Results go to an LDS tile [64 pixels][depth chunk * C] (row stride
// padded to an odd word count: conflict-free 4-B writes) and leave as coalesced
// 4-B stores along each pixel's output run -- for the bare volume the whole tile is
// one contiguous run.  Depths are processed in chunks of kTileD so the LDS tile
// stays <= 64 KiB; the 4 waves take interleaved depths, kSweepDG at a time.
constexpr int kTileP = 64;  // pixels per block (one per lane)
constexpr int kTileD = 64;  // depths per LDS chunk

template <int C>
__global__ __launch_bounds__(256) void plane_sweep_tile_kernel(const float4* __restrict__ img4, SweepParams sp,
                                                               PadGeom pg, float rc_hs, float rc_ws, FastDiv fd_w,
                                                               FastDiv fd_run_full, FastDiv fd_run_last,
                                                               const float* __restrict__ ki,
                                                               const float* __restrict__ proj,
                                                               const float* __restrict__ depths,
                                                               float* __restrict__ out, int64_t out_bstride,
                                                               int64_t out_pstride) {
    constexpr int RS = kTileD * C + 1;  // LDS row stride (words): odd -> conflict-free lane-per-row writes
    __shared__ float s_tile[kTileP * RS];
    const int npix = sp.Ht * sp.Wt;
    const int pix0 = blockIdx.x * kTileP;
    const int b = blockIdx.y;
    const int lane = threadIdx.x & (kWave - 1), wave = threadIdx.x >> 6;
    const int pix = min(pix0 + lane, npix - 1);  // tail lanes recompute the last pixel
    const unsigned yy = fast_div((unsigned)pix, fd_w);
    const float fy = (float)(int)yy, fx = (float)(int)(pix - yy * sp.Wt);
    const float* m = proj + (int64_t)b * 16;
    float rx, ry, rz;
    ray(ki + (int64_t)b * 9, fx, fy, rx, ry, rz);  // pixel2cam_torch, utils.py:370
    const __amdgpu_buffer_rsrc_t r = make_rsrc(img4 + (int64_t)b * pg.plane_bytes / 16, pg.plane_bytes);
    const int np = min(kTileP, npix - pix0);
    float* ob = out + (int64_t)b * out_bstride;

    for (int dc0 = 0; dc0 < sp.D; dc0 += kTileD) {
        const int nd = min(kTileD, sp.D - dc0);
        // wave w: depths dc0 + w + 4*i, kSweepDG of them per step
        for (int i0 = 0; i0 * 4 + wave < nd; i0 += kSweepDG) {
            TapSet t[kSweepDG];
#pragma unroll
            for (int j = 0; j < kSweepDG; ++j) {
                const int dl = min((i0 + j) * 4 + wave, nd - 1);
                const float dep = depths[dc0 + dl];
                const float X = rx * dep, Y = ry * dep, Z = rz * dep;
                const float pu = __builtin_fmaf(m[2], Z, __builtin_fmaf(m[1], Y, m[0] * X)) + m[3];
                const float pv = __builtin_fmaf(m[6], Z, __builtin_fmaf(m[5], Y, m[4] * X)) + m[7];
                const float pz = __builtin_fmaf(m[10], Z, __builtin_fmaf(m[9], Y, m[8] * X)) + m[11];
                float su, sv;
                div2_rn(pu, pv, pz + 1e-10f, su, sv);  // cam2pixel_torch, utils.py:388-391
                const float cx = div_const(su + 0.5f, sp.fhs, rc_hs);  // SWAPPED: x / H, utils.py:444
                const float cy = div_const(sv + 0.5f, sp.fws, rc_ws);  //          y / W
                issue_taps_padded(r, sp.Ws, sp.Hs, pg.Wp, pg.org, pg.row, unnormalize(to_grid(cx), sp.half_ws),
                                  unnormalize(to_grid(cy), sp.half_hs), t[j]);
            }
#pragma unroll
            for (int j = 0; j < kSweepDG; ++j) {
                const int dl = (i0 + j) * 4 + wave;
                const f32x4 v = blend_taps(t[j]);
                if (dl < nd) {
#pragma unroll
                    for (int c = 0; c < C; ++c) s_tile[lane * RS + dl * C + c] = v[c];
                }
            }
        }
        __syncthreads();
        // write out: per pixel a run of nd*C floats at pix*out_pstride + dc0*C
        const int run = nd * C;
        const int total = np * run;
        const FastDiv fd_run = nd == kTileD ? fd_run_full : fd_run_last;  // divides by run
        for (int k = threadIdx.x; k < total; k += blockDim.x) {
            const int p = (int)fast_div((unsigned)k, fd_run);
            const int e = k - p * run;
            ob[(int64_t)(pix0 + p) * out_pstride + dc0 * C + e] = s_tile[p * RS + e];
        }
        __syncthreads();
    }
}

// depth `dep` along a camera ray -> source sample position, the fast exact form of
// sweep_pos (u/den and v/den share one reciprocal, the two launch-constant divisions use
// div_const); den = pz + 1e-10 is returned for the LDS sweep's sign test
__device__ __forceinline__ void sweep_pos_fast(const float* __restrict__ m, float rx, float ry, float rz,
                                               float dep, const SweepParams& sp, float rc_hs, float rc_ws,
                                               float& px, float& py, float& den) {
    const float X = rx * dep, Y = ry * dep, Z = rz * dep;
    const float pu = __builtin_fmaf(m[2], Z, __builtin_fmaf(m[1], Y, m[0] * X)) + m[3];
    const float pv = __builtin_fmaf(m[6], Z, __builtin_fmaf(m[5], Y, m[4] * X)) + m[7];
    const float pz = __builtin_fmaf(m[10], Z, __builtin_fmaf(m[9], Y, m[8] * X)) + m[11];
    den = pz + 1e-10f;
    float su, sv;
    div2_rn(pu, pv, den, su, sv);  // cam2pixel_torch, utils.py:388-391
    const float cx = div_const(su + 0.5f, sp.fhs, rc_hs);  // SWAPPED: x / H, utils.py:444
    const float cy = div_const(sv + 0.5f, sp.fws, rc_ws);  //          y / W
    px = unnormalize(to_grid(cx), sp.half_ws);
    py = unnormalize(to_grid(cy), sp.half_hs);
}

// LDS-staged sweep (the default for C <= 4, D <= kSweepMaxLdsD).  A block owns a tile of
// kSLR target rows x kSLP pixels of one view and sweeps it through ALL depths, so each of
// its row segments is one contiguous run of the volume (np * D * C floats for the bare
// volume).  Its source footprint is small and known up front: cam2pixel's homogeneous
// point (pu, pv, pz) is affine in x, in y and in the depth separately, so while
// pz + 1e-10 keeps its sign -- trilinear, so its 8 vertex values decide -- every sample
// of the tile lies in the convex hull of the images of the 8 vertices (x first | last) x
// (row first | last) x (depth min | max): for a fixed depth the tile maps by a homography
// onto the hull of its corners, for a fixed pixel the depths map onto a segment.  The box
// [floor(min) - 1, floor(max) + 2] of the 8 computed vertex positions (render_lds.hip's
// margin argument) is staged in LDS once, and the tile's samples read their taps there:
// the vector-L1 tap traffic (64 B per sample, what bounds the global-gather kernels
// above) shrinks to one box fill per block.  A sample whose tap origin is not staged
// (image borders, rounding at ill-conditioned geometry, NaN) is gathered from global
// memory (lds_sample), and a block whose box is invalid or too large gathers everything
// from global memory: the output is bit-identical whatever the geometry.
//
// Stores: a lane's kSweepDG*C results are one 16*C-byte piece and a wave's 64 pieces are
// one contiguous run of the bare volume, but 16-B stores at a 16*C-byte lane stride
// reach the L2 as ~C times more, partial, write requests (measured 4x the tile kernel's).
// So a wave whose 64 groups are complete and dense passes its pieces through a per-wave
// LDS slot and stores the run with lane-contiguous 16-B stores.
constexpr int kSLP = 64;                           // target pixels per tile row
#ifndef MPIV_SLR
#define MPIV_SLR 4
#endif
#ifndef MPIV_SLCAP
#define MPIV_SLCAP 3072
#endif
constexpr int kSLR = MPIV_SLR;                     // target rows per tile
constexpr int kSLThreads = 512;                    // 8 waves
constexpr int kSLCap = MPIV_SLCAP;                 // staged source texels (48 KiB; 2 blocks per CU)
constexpr int kSLFill = kSLCap / kSLThreads;       // staged texels per thread

// wave-scope LDS ordering: every lane's LDS stores before any lane's later loads
__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// C <= 3 must keep 4 waves per SIMD (two 512-thread blocks per CU, which the LDS allows):
// the register allocator otherwise lands a few VGPRs above 128 and halves the occupancy.
template <int C>
__global__ __launch_bounds__(kSLThreads) __attribute__((amdgpu_waves_per_eu(C <= 3 ? 4 : 1))) void plane_sweep_lds_kernel(
    const float4* __restrict__ img4, SweepParams sp, PadGeom pg, float rc_hs, float rc_ws, FastDiv fd_g,
    FastDiv fd_b, const float* __restrict__ ki, const float* __restrict__ proj, const float* __restrict__ depths,
    float* __restrict__ out, int64_t out_bstride, int64_t out_pstride, int vec, int shrink) {
    constexpr int kWaves = kSLThreads / kWave;
    __shared__ __attribute__((aligned(16))) float4 s_src[kSLCap];
    __shared__ __attribute__((aligned(16))) float s_dep[kSweepMaxLdsD];
    __shared__ int4 s_box;              // x_lo, y_lo, rows, pitch (0: gather from global memory)
    __shared__ int s_fast;              // every sample of the tile is in div2_rn's fast range
    __shared__ int s_zero;              // every tap of the tile lies outside the source image
    __shared__ __attribute__((aligned(16))) float4 s_out[kWaves][kWave * C];  // per wave: its run

    const int segs = (sp.Wt + kSLP - 1) / kSLP;
    const int b = blockIdx.y;
    const int ty = blockIdx.x / segs;
    const int y0 = ty * kSLR, x0 = (blockIdx.x - ty * segs) * kSLP;
    const int np = min(kSLP, sp.Wt - x0), nr = min(kSLR, sp.Ht - y0);
    const int lane = threadIdx.x & (kWave - 1), wave = threadIdx.x >> 6;
    const float* k9 = ki + (int64_t)b * 9;
    const float* m = proj + (int64_t)b * 16;
    const __amdgpu_buffer_rsrc_t r = make_rsrc(img4 + (int64_t)b * (pg.plane_bytes / 16), pg.plane_bytes);

    // depths -> LDS (all threads); wave 0 also reduces their range itself, so the box
    // prologue needs no block barrier before the vertex computation
    for (int i = threadIdx.x; i < sp.D; i += kSLThreads) s_dep[i] = depths[i];
    if (wave == 0) {  // vertex = lane % 8: (first | last pixel) x (first | last row) x (min | max depth)
        float dmin = __builtin_inff(), dmax = -__builtin_inff(), dbad = 0.0f;
        for (int i = lane; i < sp.D; i += kWave) {
            const float d = depths[i];
            dmin = fminf(dmin, d);
            dmax = fmaxf(dmax, d);
            dbad = __builtin_isfinite(d) ? dbad : 1.0f;
        }
#pragma unroll
        for (int k = 1; k < kWave; k <<= 1) {
            dmin = fminf(dmin, __shfl_xor(dmin, k));
            dmax = fmaxf(dmax, __shfl_xor(dmax, k));
            dbad = fmaxf(dbad, __shfl_xor(dbad, k));
        }
        const int vtx = lane & 7;
        float rx, ry, rz;
        ray(k9, (float)((vtx & 1) ? x0 + np - 1 : x0), (float)((vtx & 2) ? y0 + nr - 1 : y0), rx, ry, rz);
        float px, py, den;
        sweep_pos_fast(m, rx, ry, rz, (vtx & 4) ? dmax : dmin, sp, rc_hs, rc_ws, px, py, den);
        // pu, pv and den are multi-affine in (x, y, depth): over the tile their extremes are
        // at the 8 vertices, so vertex values a factor 2 inside div2_safe's range (room for
        // rounding) prove the fast division exact for every sample of the tile
        const float dep = (vtx & 4) ? dmax : dmin;
        const float X = rx * dep, Y = ry * dep, Z = rz * dep;
        const float pu = __builtin_fmaf(m[2], Z, __builtin_fmaf(m[1], Y, m[0] * X)) + m[3];
        const float pv = __builtin_fmaf(m[6], Z, __builtin_fmaf(m[5], Y, m[4] * X)) + m[7];
        const float ad = __builtin_fabsf(den);
        int fastv = ad >= 0x1p-59f && ad <= 0x1p59f && __builtin_fmaxf(__builtin_fabsf(pu), __builtin_fabsf(pv)) <= 0x1p59f;
        const bool fin = dbad == 0.0f && __builtin_isfinite(px) && __builtin_isfinite(py) &&
                         __builtin_fabsf(px) < 1e7f && __builtin_fabsf(py) < 1e7f;
        float xmin = floorf(px), xmax = xmin, ymin = floorf(py), ymax = ymin;
        int pos = fin && den > 0.0f, neg = fin && den < 0.0f;
#pragma unroll
        for (int k = 1; k < 8; k <<= 1) {
            xmin = fminf(xmin, __shfl_xor(xmin, k));
            xmax = fmaxf(xmax, __shfl_xor(xmax, k));
            ymin = fminf(ymin, __shfl_xor(ymin, k));
            ymax = fmaxf(ymax, __shfl_xor(ymax, k));
            pos &= __shfl_xor(pos, k);
            neg &= __shfl_xor(neg, k);
            fastv &= __shfl_xor(fastv, k);
        }
        if (lane == 0) {
            const bool ok = pos || neg;
            s_fast = ok && fin && fastv;
            int xl = ok ? max((int)xmin - 1 + shrink, -2) : 0;
            int xh = ok ? min((int)xmax + 2 - shrink, sp.Ws + 1) : 0;
            int yl = ok ? max((int)ymin - 1 + shrink, -2) : 0;
            int yh = ok ? min((int)ymax + 2 - shrink, sp.Hs + 1) : 0;
            // A footprint wholly beyond one side of the image (the reference's swapped
            // x / H normalisation sends every sample past x = 3W/4 out of a landscape
            // source) stages the 3 columns (rows) at that edge: origins past the edge are
            // then read exactly as the border's zeros (LdsBox's open border edges), so
            // these tiles stay on the LDS path instead of gathering zeros from memory.
            if (ok && xl > xh) {
                xl = xh == sp.Ws + 1 ? sp.Ws - 1 : -2;
                xh = xl + 2;
            }
            if (ok && yl > yh) {
                yl = yh == sp.Hs + 1 ? sp.Hs - 1 : -2;
                yh = yl + 2;
            }
            const int width = xh - xl + 1, rows = yh - yl + 1;
            const bool fits = ok && width >= 2 && rows >= 2 && width <= kSLCap && rows <= kSLCap &&
                              width * rows <= kSLCap;
            s_box = make_int4(xl, yl, rows, fits ? width : 0);
            // Every tap of every sample outside the image: each sample is a blend of four
            // zero texels with finite non-negative weights, i.e. exactly +0.  Interior
            // samples lie in the hull of the 8 vertex positions (the box argument above) up
            // to rounding far below the one-texel margin while |coordinates| < 2^16.
            const bool small = xmin > -65536.0f && xmax < 65536.0f && ymin > -65536.0f && ymax < 65536.0f;
            s_zero = ok && small && shrink == 0 &&
                     ((int)xmin - 1 >= sp.Ws || (int)xmax + 2 <= -1 || (int)ymin - 1 >= sp.Hs || (int)ymax + 2 <= -1);
        }
    }
    __syncthreads();
    if (__builtin_amdgcn_readfirstlane(s_zero)) {  // the tile's output is all +0: store it
        const int64_t run = (int64_t)np * sp.D * C;
        for (int tr = 0; tr < nr; ++tr) {
            float* ob = out + (int64_t)b * out_bstride + ((int64_t)(y0 + tr) * sp.Wt + x0) * out_pstride;
            if (vec && out_pstride == (int64_t)sp.D * C && run % 4 == 0) {  // one dense 16-B-aligned run
                f32x4* o4 = reinterpret_cast<f32x4*>(ob);
                const f32x4 z = {0.f, 0.f, 0.f, 0.f};
                for (int64_t i = threadIdx.x; i < run / 4; i += kSLThreads) __builtin_nontemporal_store(z, o4 + i);
            } else {
                for (int64_t i = threadIdx.x; i < run; i += kSLThreads) {
                    const int pxl = (int)(i / (sp.D * C)), e = (int)(i - (int64_t)pxl * sp.D * C);
                    ob[(int64_t)pxl * out_pstride + e] = 0.0f;
                }
            }
        }
        return;
    }
    const int xl = __builtin_amdgcn_readfirstlane(s_box.x), yl = __builtin_amdgcn_readfirstlane(s_box.y);
    const int rows = __builtin_amdgcn_readfirstlane(s_box.z), pitch = __builtin_amdgcn_readfirstlane(s_box.w);
    const bool all_fast = __builtin_amdgcn_readfirstlane(s_fast) != 0;
    if (pitch > 0) {  // fill: box texel idx = row * pitch + col <- padded-plane texel
        const int nfp = rows * pitch;
        const float rp = 1.0f / (float)pitch;
        const int org = (yl + kPad) * pg.Wp + xl + kPad;  // >= 0: boxes start at -2
        f32x4 stg[kSLFill];
#pragma unroll
        for (int k = 0; k < kSLFill; ++k) {
            if (kSLThreads * k < nfp) {
                const int idx = threadIdx.x + kSLThreads * k;
                int row = (int)((float)idx * rp);  // idx < 2^12: off by at most one, corrected
                row -= row * pitch > idx ? 1 : 0;
                row += (row + 1) * pitch <= idx ? 1 : 0;
                stg[k] = llvm_raw_buffer_load_v4f32(r, (org + row * pg.Wp + idx - row * pitch) * 16, 0, 0);
            }
        }
#pragma unroll
        for (int k = 0; k < kSLFill; ++k)
            if (kSLThreads * k < nfp) *reinterpret_cast<f32x4*>(&s_src[threadIdx.x + kSLThreads * k]) = stg[k];
    }
    __syncthreads();

    // samples: item group g -> (tile row g / (np*NG); pixel, depths kSweepDG*dg ...), groups fastest
    const int NG = (sp.D + kSweepDG - 1) / kSweepDG;
    const int nrow = np * NG;  // groups per tile row
    const int ngr = nr * nrow;
    const LdsBox lbx = make_lds_box(xl, yl, rows, pitch, sp.Ws, sp.Hs);
    // every group complete and pixels packed: each tile row's output is one dense run
    const bool d4 = sp.D % kSweepDG == 0;  // whole depth groups: one 16-B LDS read per group
    const bool dense = vec && d4 && out_pstride == (int64_t)sp.D * C;
    // Pixel-interleaved order (when the tile row splits into whole 16-pixel blocks and
    // the depth groups into fours): a wave takes 16 consecutive pixels x 4 consecutive
    // depth groups, pixel fastest, so each 8-lane phase of a tap read touches ~8
    // consecutive staged texels (one depth, neighbouring pixels) instead of 8 points
    // along one pixel's epipolar line -- no LDS bank conflicts.  Each pixel's 4 groups are
    // one 16C-float piece of its run, so the wave's output is 16 whole 64-B-aligned pieces.
    const bool pix16 = np % 16 == 0 && NG % 4 == 0;
    const int nb16 = 16 * NG;  // groups per 16-pixel block
    int lane_off[C];           // dense pixel-interleaved stores: float4 offsets of this lane's
#pragma unroll                 // k-th store in the wave's 16 pieces
    for (int k = 0; k < C; ++k) {
        const int f = k * kWave + lane;
        const int pc = f / (4 * C), qc = f - pc * 4 * C;
        lane_off[k] = pc * (sp.D * C / 4) + qc;
    }
    // The per-wave slot in that order: lane (pixel pq, group dq) writes its k-th float4 at
    // pq*4C + dq*C + k and lane l reads float4 k*64 + l.  ds_*_b128 serve 16 lanes per pass
    // over 16 16-B bank slots, and the writes of one pass (pq = 0..15) fall on 4 slots (C = 1,
    // 3) or 1 (C = 4): up to 16-way conflicts.  Rotating each 16-float4 row a of the slot by
    // G(a) (a / 3 for C = 3, a otherwise; a bijection within the row) makes both the write
    // and the read passes conflict-free (checked for C = 1..4 by enumeration).
    auto swz = [](int L) { return (L & ~15) | ((L + (C == 3 ? (L >> 4) / 3 : (L >> 4))) & 15); };
    int so_w[C], so_r[C];  // lane constants: swizzled write / read slots
#pragma unroll
    for (int k = 0; k < C; ++k) {
        so_w[k] = swz((lane & 15) * 4 * C + (lane >> 4) * C + k);
        so_r[k] = swz(k * kWave + lane);
    }
#ifndef MPIV_SWEEP_HOIST
#define MPIV_SWEEP_HOIST 1
#endif
    // When the thread stride is a multiple of the 16-pixel block's groups (D = 64: 256
    // groups), a thread's depth group is the same in every iteration: its 4 depths are read
    // from LDS once, not once per iteration (one LDS round trip fewer per iteration).
    const bool hoist = MPIV_SWEEP_HOIST && pix16 && d4 && kSLThreads % nb16 == 0;
    f32x4 dqh = {0.f, 0.f, 0.f, 0.f};
    if (hoist) dqh = *reinterpret_cast<const f32x4*>(&s_dep[((threadIdx.x % nb16) >> 4) * kSweepDG]);
    for (int gi = threadIdx.x; gi < ngr; gi += kSLThreads) {
        int tr = 0;  // tile row of group gi
#pragma unroll
        for (int k = 1; k < kSLR; ++k) tr += gi >= k * nrow ? 1 : 0;
        const int gr = gi - tr * nrow;
        int pl, dg;
        if (pix16) {
            const int blk = (int)fast_div((unsigned)gr, fd_b), rem = gr - blk * nb16;
            dg = rem >> 4;
            pl = blk * 16 + (rem & 15);
        } else {
            pl = (int)fast_div((unsigned)gr, fd_g);
            dg = gr - pl * NG;
        }
        float* ob = out + (int64_t)b * out_bstride + ((int64_t)(y0 + tr) * sp.Wt + x0) * out_pstride;
        float rx, ry, rz;
        ray(k9, (float)(x0 + (int)pl), (float)(y0 + tr), rx, ry, rz);  // pixel2cam_torch, utils.py:370
        // The kSweepDG samples run phase by phase (all positions, all tap reads, all
        // blends) with the rare fix-ups behind wave-uniform tests, so their LDS reads are
        // in flight together instead of one round trip per sample.
        float su[kSweepDG], sv[kSweepDG], dq[kSweepDG];
        if (hoist) {
#pragma unroll
            for (int j = 0; j < kSweepDG; ++j) dq[j] = dqh[j];
        } else if (d4) {
            const f32x4 q = *reinterpret_cast<const f32x4*>(&s_dep[dg * kSweepDG]);
#pragma unroll
            for (int j = 0; j < kSweepDG; ++j) dq[j] = q[j];
        } else {
#pragma unroll
            for (int j = 0; j < kSweepDG; ++j) dq[j] = s_dep[min(dg * kSweepDG + j, sp.D - 1)];  // partial group: D-1
        }
        bool fast = true;
#pragma unroll
        for (int j = 0; j < kSweepDG; ++j) {
            const float dep = dq[j];
            const float X = rx * dep, Y = ry * dep, Z = rz * dep;
            const float pu = __builtin_fmaf(m[2], Z, __builtin_fmaf(m[1], Y, m[0] * X)) + m[3];
            const float pv = __builtin_fmaf(m[6], Z, __builtin_fmaf(m[5], Y, m[4] * X)) + m[7];
            const float den = __builtin_fmaf(m[10], Z, __builtin_fmaf(m[9], Y, m[8] * X)) + m[11] + 1e-10f;
            if (!all_fast) fast = fast && div2_safe(pu, pv, den);
            div2_fast(pu, pv, den, su[j], sv[j]);  // cam2pixel_torch, utils.py:388-391
        }
        if (__builtin_amdgcn_ballot_w64(!fast)) {  // rare: a quotient outside the fast path's range
#pragma unroll
            for (int j = 0; j < kSweepDG; ++j) {
                const float dep = dq[j];
                const float X = rx * dep, Y = ry * dep, Z = rz * dep;
                const float pu = __builtin_fmaf(m[2], Z, __builtin_fmaf(m[1], Y, m[0] * X)) + m[3];
                const float pv = __builtin_fmaf(m[6], Z, __builtin_fmaf(m[5], Y, m[4] * X)) + m[7];
                const float den = __builtin_fmaf(m[10], Z, __builtin_fmaf(m[9], Y, m[8] * X)) + m[11] + 1e-10f;
                if (!div2_safe(pu, pv, den)) {
                    su[j] = div_rn(pu, den);
                    sv[j] = div_rn(pv, den);
                }
            }
        }
        float px[kSweepDG], py[kSweepDG];
#pragma unroll
        for (int j = 0; j < kSweepDG; ++j) {
            const float cx = div_const(su[j] + 0.5f, sp.fhs, rc_hs);  // SWAPPED: x / H, utils.py:444
            const float cy = div_const(sv[j] + 0.5f, sp.fws, rc_ws);  //          y / W
            px[j] = unnormalize(to_grid(cx), sp.half_ws);
            py[j] = unnormalize(to_grid(cy), sp.half_hs);
        }
        f32x4 s[kSweepDG];
        bool staged = pitch > 0;
#ifndef MPIV_SWEEP_B128
#define MPIV_SWEEP_B128 1
#endif
        if (MPIV_SWEEP_B128 && staged && C == 3) {
            // RGB through 16-B tap reads (ds_read_b128: 4 LDS cycles per wave read,
            // ds_read_b96: 8), at most 12 in flight: depth 3's taps are issued into the
            // registers depth 0's blend frees
            TapSet ts[kSweepDG];
#pragma unroll
            for (int j = 0; j < 3; ++j) staged = lds_issue(s_src, lbx, px[j], py[j], ts[j]) && staged;
            s[0] = blend_taps3(TapSet3{ts[0].a.xyz, ts[0].b.xyz, ts[0].c.xyz, ts[0].d.xyz, ts[0].nw, ts[0].ne,
                                       ts[0].sw, ts[0].se});
            asm volatile("" ::"v"(ts[0].a), "v"(ts[0].b), "v"(ts[0].c), "v"(ts[0].d));
            staged = lds_issue(s_src, lbx, px[3], py[3], ts[3]) && staged;
#pragma unroll
            for (int j = 1; j < kSweepDG; ++j)
                s[j] = blend_taps3(TapSet3{ts[j].a.xyz, ts[j].b.xyz, ts[j].c.xyz, ts[j].d.xyz, ts[j].nw, ts[j].ne,
                                           ts[j].sw, ts[j].se});
            // the dead 4th channels keep their registers until the reads are consumed (else a
            // WAW wait serialises the reads, as in the C < 4 path below)
#pragma unroll
            for (int j = 1; j < kSweepDG; ++j)
                asm volatile("" ::"v"(ts[j].a), "v"(ts[j].b), "v"(ts[j].c), "v"(ts[j].d));
        } else if (staged && C == 3) {  // RGB: 12-B tap reads, 3-channel blends
            TapSet3 ts[kSweepDG];
#pragma unroll
            for (int j = 0; j < kSweepDG; ++j) staged = lds_issue3(s_src, lbx, px[j], py[j], ts[j]) && staged;
#pragma unroll
            for (int j = 0; j < kSweepDG; ++j) s[j] = blend_taps3(ts[j]);
        } else if (staged) {
            TapSet ts[kSweepDG];
#pragma unroll
            for (int j = 0; j < kSweepDG; ++j) staged = lds_issue(s_src, lbx, px[j], py[j], ts[j]) && staged;
#pragma unroll
            for (int j = 0; j < kSweepDG; ++j) s[j] = blend_taps(ts[j]);
            // keep every tap register live until here: for C < 4 the unused channels are
            // dead, and hipcc otherwise reuses those registers while the reads are still in
            // flight (a WAW wait after each pair of reads serialises the LDS round trips)
#pragma unroll
            for (int j = 0; j < kSweepDG; ++j)
                asm volatile("" ::"v"(ts[j].a), "v"(ts[j].b), "v"(ts[j].c), "v"(ts[j].d));
        }
        if (__builtin_amdgcn_ballot_w64(!staged)) {  // wave-uniform test, then per lane
            if (!staged) {                            // a tap origin not staged: gather from global memory
                TapSet ts[kSweepDG];
#pragma unroll
                for (int j = 0; j < kSweepDG; ++j)
                    issue_taps_padded(r, sp.Ws, sp.Hs, pg.Wp, pg.org, pg.row, px[j], py[j], ts[j]);
#pragma unroll
                for (int j = 0; j < kSweepDG; ++j) s[j] = blend_taps(ts[j]);
            }
        }
        float v[kSweepDG * C];
#pragma unroll
        for (int j = 0; j < kSweepDG; ++j)
#pragma unroll
            for (int c = 0; c < C; ++c) v[j * C + c] = s[j][c];
        // the wave's first group, and its offset in that group's tile row (wave-uniform)
        const int gw = __builtin_amdgcn_readfirstlane(gi - lane);
        int g0 = gw;
#pragma unroll
        for (int k = 1; k < kSLR; ++k) g0 -= gw >= k * nrow ? nrow : 0;
        if (pix16 && dense) {  // 16 pixels x 4 groups: 16 pieces of 16C floats
            float4* so = s_out[wave];
            wave_lds_sync();  // the previous iteration's reads of the slot are done
#pragma unroll
            for (int k = 0; k < C; ++k)
                so[so_w[k]] = make_float4(v[4 * k], v[4 * k + 1], v[4 * k + 2], v[4 * k + 3]);
            wave_lds_sync();
            const int blk0 = g0 / nb16, dg0 = (g0 - blk0 * nb16) >> 4;  // wave-uniform
            f32x4* base = reinterpret_cast<f32x4*>(ob + (int64_t)blk0 * 16 * out_pstride) + dg0 * C;
            const f32x4* sn = reinterpret_cast<const f32x4*>(so);
#pragma unroll
            for (int k = 0; k < C; ++k) __builtin_nontemporal_store(sn[so_r[k]], base + lane_off[k]);
        } else if (dense && g0 + kWave <= nrow) {  // all 64 groups in one tile row
            // the wave's 64 pieces are the contiguous run ob[g0*4C .. (g0+64)*4C): through
            // LDS, then lane-contiguous 16-B stores
            float4* so = s_out[wave];
            wave_lds_sync();  // the previous iteration's reads of the slot are done
#pragma unroll
            for (int k = 0; k < C; ++k)
                so[lane * C + k] = make_float4(v[4 * k], v[4 * k + 1], v[4 * k + 2], v[4 * k + 3]);
            wave_lds_sync();
            float4* run = reinterpret_cast<float4*>(ob + (int64_t)g0 * kSweepDG * C);
            // non-temporal: the volume is written once and never re-read here (measured -8 %)
            f32x4* rn = reinterpret_cast<f32x4*>(run);
            const f32x4* sn = reinterpret_cast<const f32x4*>(so);
#pragma unroll
            for (int k = 0; k < C; ++k) __builtin_nontemporal_store(sn[k * kWave + lane], &rn[k * kWave + lane]);
        } else {
            float* o = ob + (int64_t)pl * out_pstride + dg * kSweepDG * C;
            if (vec && (dg + 1) * kSweepDG <= sp.D) {
#pragma unroll
                for (int k = 0; k < C; ++k)  // kSweepDG * C floats = C float4
                    reinterpret_cast<float4*>(o)[k] =
                        make_float4(v[4 * k], v[4 * k + 1], v[4 * k + 2], v[4 * k + 3]);
            } else {
                const int nd = min(kSweepDG, sp.D - dg * kSweepDG);
#pragma unroll
                for (int j = 0; j < kSweepDG; ++j)
                    if (j < nd)
#pragma unroll
                        for (int c = 0; c < C; ++c) o[j * C + c] = v[j * C + c];
            }
        }
    }
}

// Depth range of the sweep, reduced by one wave: min, max, and whether any depth is not
// finite (every lane gets the result).
__device__ __forceinline__ void sweep_depth_range(const float* __restrict__ depths, int D, int lane, float& dmin,
                                                  float& dmax, float& dbad) {
    dmin = __builtin_inff();
    dmax = -__builtin_inff();
    dbad = 0.0f;
    for (int i = lane; i < D; i += kWave) {
        const float d = depths[i];
        dmin = fminf(dmin, d);
        dmax = fmaxf(dmax, d);
        dbad = __builtin_isfinite(d) ? dbad : 1.0f;
    }
#pragma unroll
    for (int k = 1; k < kWave; k <<= 1) {
        dmin = fminf(dmin, __shfl_xor(dmin, k));
        dmax = fmaxf(dmax, __shfl_xor(dmax, k));
        dbad = fmaxf(dbad, __shfl_xor(dbad, k));
    }
}

// A tile's staged source box and its two flags, computed by one wave (lanes 0..7 are the
// 8 vertices; lane 0 holds the result).
struct SweepBox {
    int xl, yl, rows, pitch;  // pitch 0: gather every sample from global memory
    int fast;                 // every sample of the tile is in div2_rn's fast range
    int zero;                 // every tap of the tile lies outside the source image
};

__device__ __forceinline__ SweepBox sweep_tile_box(const float* __restrict__ k9, const float* __restrict__ m,
                                                   const SweepParams& sp, float rc_hs, float rc_ws, int x0, int y0,
                                                   int np, int nr, float dmin, float dmax, float dbad, int shrink,
                                                   int lane, int cap = kSLCap) {
    // vertex = lane % 8: (first | last pixel) x (first | last row) x (min | max depth)
    const int vtx = lane & 7;
    float rx, ry, rz;
    ray(k9, (float)((vtx & 1) ? x0 + np - 1 : x0), (float)((vtx & 2) ? y0 + nr - 1 : y0), rx, ry, rz);
    float px, py, den;
    sweep_pos_fast(m, rx, ry, rz, (vtx & 4) ? dmax : dmin, sp, rc_hs, rc_ws, px, py, den);
    // pu, pv and den are multi-affine in (x, y, depth): over the tile their extremes are
    // at the 8 vertices, so vertex values a factor 2 inside div2_safe's range (room for
    // rounding) prove the fast division exact for every sample of the tile
    const float dep = (vtx & 4) ? dmax : dmin;
    const float X = rx * dep, Y = ry * dep, Z = rz * dep;
    const float pu = __builtin_fmaf(m[2], Z, __builtin_fmaf(m[1], Y, m[0] * X)) + m[3];
    const float pv = __builtin_fmaf(m[6], Z, __builtin_fmaf(m[5], Y, m[4] * X)) + m[7];
    const float ad = __builtin_fabsf(den);
    int fastv = ad >= 0x1p-59f && ad <= 0x1p59f && __builtin_fmaxf(__builtin_fabsf(pu), __builtin_fabsf(pv)) <= 0x1p59f;
    const bool fin = dbad == 0.0f && __builtin_isfinite(px) && __builtin_isfinite(py) && __builtin_fabsf(px) < 1e7f &&
                     __builtin_fabsf(py) < 1e7f;
    float xmin = floorf(px), xmax = xmin, ymin = floorf(py), ymax = ymin;
    int pos = fin && den > 0.0f, neg = fin && den < 0.0f;
#pragma unroll
    for (int k = 1; k < 8; k <<= 1) {
        xmin = fminf(xmin, __shfl_xor(xmin, k));
        xmax = fmaxf(xmax, __shfl_xor(xmax, k));
        ymin = fminf(ymin, __shfl_xor(ymin, k));
        ymax = fmaxf(ymax, __shfl_xor(ymax, k));
        pos &= __shfl_xor(pos, k);
        neg &= __shfl_xor(neg, k);
        fastv &= __shfl_xor(fastv, k);
    }
    SweepBox bx;
    const bool ok = pos || neg;
    bx.fast = ok && fin && fastv;
    int xl = ok ? max((int)xmin - 1 + shrink, -2) : 0;
    int xh = ok ? min((int)xmax + 2 - shrink, sp.Ws + 1) : 0;
    int yl = ok ? max((int)ymin - 1 + shrink, -2) : 0;
    int yh = ok ? min((int)ymax + 2 - shrink, sp.Hs + 1) : 0;
    // A footprint wholly beyond one side of the image (the reference's swapped x / H
    // normalisation sends every sample past x = 3W/4 out of a landscape source) stages the
    // 3 columns (rows) at that edge: origins past the edge are then read exactly as the
    // border's zeros (LdsBox's open border edges), so these tiles stay on the LDS path
    // instead of gathering zeros from memory.
    if (ok && xl > xh) {
        xl = xh == sp.Ws + 1 ? sp.Ws - 1 : -2;
        xh = xl + 2;
    }
    if (ok && yl > yh) {
        yl = yh == sp.Hs + 1 ? sp.Hs - 1 : -2;
        yh = yl + 2;
    }
    const int width = xh - xl + 1, rows = yh - yl + 1;
    const bool fits = ok && width >= 2 && rows >= 2 && width <= cap && rows <= cap && width * rows <= cap;
    bx.xl = xl;
    bx.yl = yl;
    bx.rows = rows;
    bx.pitch = fits ? width : 0;
    // Every tap of every sample outside the image: each sample is a blend of four zero
    // texels with finite non-negative weights, i.e. exactly +0.  Interior samples lie in
    // the hull of the 8 vertex positions (the box argument above) up to rounding far below
    // the one-texel margin while |coordinates| < 2^16.
    const bool small = xmin > -65536.0f && xmax < 65536.0f && ymin > -65536.0f && ymax < 65536.0f;
    bx.zero = ok && small && shrink == 0 &&
              ((int)xmin - 1 >= sp.Ws || (int)xmax + 2 <= -1 || (int)ymin - 1 >= sp.Hs || (int)ymax + 2 <= -1);
    return bx;
}

// The all-+0 output of a zero tile (NT threads of the block).
template <int C, int NT>
__device__ __forceinline__ void sweep_zero_tile(float* __restrict__ out, int64_t out_bstride, int64_t out_pstride,
                                                const SweepParams& sp, int vec, int b, int x0, int y0, int np,
                                                int nr) {
    const int64_t run = (int64_t)np * sp.D * C;
    for (int tr = 0; tr < nr; ++tr) {
        float* ob = out + (int64_t)b * out_bstride + ((int64_t)(y0 + tr) * sp.Wt + x0) * out_pstride;
        if (vec && out_pstride == (int64_t)sp.D * C && run % 4 == 0) {  // one dense 16-B-aligned run
            f32x4* o4 = reinterpret_cast<f32x4*>(ob);
            const f32x4 z = {0.f, 0.f, 0.f, 0.f};
            for (int64_t i = threadIdx.x; i < run / 4; i += NT) __builtin_nontemporal_store(z, o4 + i);
        } else {
            for (int64_t i = threadIdx.x; i < run; i += NT) {
                const int pxl = (int)(i / (sp.D * C)), e = (int)(i - (int64_t)pxl * sp.D * C);
                ob[(int64_t)pxl * out_pstride + e] = 0.0f;
            }
        }
    }
}

// Register-staged box fill (the non-persistent kernel): box texel idx = row * pitch + col
// <- padded-plane texel.
template <int NT, int CAP = kSLCap>
__device__ __forceinline__ void sweep_fill_box(float4* __restrict__ s_src, __amdgpu_buffer_rsrc_t r,
                                               const PadGeom& pg, const SweepBox& bx) {
    constexpr int kFill = CAP / NT;  // staged texels per thread
    const int nfp = bx.rows * bx.pitch;
    const float rp = 1.0f / (float)bx.pitch;
    const int org = (bx.yl + kPad) * pg.Wp + bx.xl + kPad;  // >= 0: boxes start at -2
    // every slot of the staging array is written (texels past the box as zeros: the
    // out-of-range buffer offset), so the loads and stores need no guards
    f32x4 stg[kFill];
#pragma unroll
    for (int k = 0; k < kFill; ++k) {
        const int idx = threadIdx.x + NT * k;
        int row = (int)((float)idx * rp);  // idx < 2^12: off by at most one, corrected
        row -= row * bx.pitch > idx ? 1 : 0;
        row += (row + 1) * bx.pitch <= idx ? 1 : 0;
        stg[k] = llvm_raw_buffer_load_v4f32(r, idx < nfp ? (org + row * pg.Wp + idx - row * bx.pitch) * 16 : kOOB,
                                            0, 0);
    }
#pragma unroll
    for (int k = 0; k < kFill; ++k) *reinterpret_cast<f32x4*>(&s_src[threadIdx.x + NT * k]) = stg[k];
}


// Depth-per-lane LDS sweep (the default when D is a multiple of 64, C <= 4).  The box
// staging is plane_sweep_lds_kernel's, but a wave's 64 lanes are the 64 depths of ONE target
// pixel (depth chunk), and it takes two pixels per iteration:
//  * a lane's depth is a register (no depth table in LDS), and the pixel's D*C-float run of
//    the volume leaves as one lane-contiguous store per 64 depths (64 x C floats): whole
//    lines, no per-wave store slot, no LDS round trip between the blend and the store;
//  * without the 24 KiB store slot and the depth table a block needs 48 KiB of LDS, so three
//    blocks fit a CU, and two samples in flight per lane keep the VGPRs under 80: 6 waves per
//    SIMD instead of 4.
// The ray of the pixel is the same in every lane (a wave-uniform VALU value).  Per sample the
// arithmetic is the same sequence as plane_sweep_lds_kernel's (bit-identical output).
#ifndef MPIV_SWNT
#define MPIV_SWNT 1  // depth-per-lane sweep: nontemporal volume stores (A/B flag)
#endif
constexpr int kDLThreads = 512;
constexpr int kDLWaves = kDLThreads / kWave;
#ifndef MPIV_DLPIX
#define MPIV_DLPIX 2
#endif
constexpr int kDLPix = MPIV_DLPIX;  // pixels (samples per lane) per iteration, D > 16 (D <= 16: 1;
                                    // profiles/r03_sweep_few_depths_ab.txt)
static_assert(kSLCap % kDLThreads == 0, "sweep_fill_box writes every staging slot");

// One source texel as a float4 (channels >= C zero), zero when !in.  Contiguous channels
// (the usual NHWC tensor) load as ONE 4*C-byte access: the fill's instruction count per texel
// matches the padded copy's 16-B loads (three scalar loads measured 0.72 vs 0.58 ms, config 3).
template <int C, bool CONTIG>
__device__ __forceinline__ f32x4 raw_texel(const float* __restrict__ t, int64_t sc, bool in) {
    f32x4 v = {0.f, 0.f, 0.f, 0.f};
    if (CONTIG) {
        typedef float f32xC __attribute__((ext_vector_type(C), aligned(4)));
        const f32xC q = *reinterpret_cast<const f32xC*>(t);
#pragma unroll
        for (int c = 0; c < C; ++c) v[c] = in ? q[c] : 0.0f;
    } else {
#pragma unroll
        for (int c = 0; c < C; ++c) v[c] = in ? t[(int64_t)c * sc] : 0.0f;
    }
    return v;
}

// RAW sources (the caller's [B,Hs,Ws,C] tensor read in place, any strides; no padded copy):
// texel (x, y) of the box is the image's where 0 <= x < Ws, 0 <= y < Hs, and zero elsewhere --
// exactly the padded buffer's values (mpiv_pad_texels writes the image inside a zero border).
// (CONTIG is decided once per fill, outside the unrolled loop: a branch per texel kept the
// loads from being in flight together)
template <int C, int NT, bool CONTIG, int CAP = kSLCap>
__device__ __forceinline__ void sweep_fill_load_raw(f32x4 (&stg)[CAP / NT], const float* __restrict__ img,
                                                    const ImgStrides& is, int Hs, int Ws, const SweepBox& bx) {
    constexpr int kFill = CAP / NT;
    const int nfp = bx.rows * bx.pitch;
    const float rp = 1.0f / (float)bx.pitch;
#pragma unroll
    for (int k = 0; k < kFill; ++k) {
        const int idx = threadIdx.x + NT * k;
        int row = (int)((float)idx * rp);  // idx < 2^12: off by at most one, corrected
        row -= row * bx.pitch > idx ? 1 : 0;
        row += (row + 1) * bx.pitch <= idx ? 1 : 0;
        const int x = bx.xl + idx - row * bx.pitch, y = bx.yl + row;
        const bool in = idx < nfp && (unsigned)x < (unsigned)Ws && (unsigned)y < (unsigned)Hs;
        const float* t = img + (in ? (int64_t)y * is.y + (int64_t)x * is.x : 0);
        stg[k] = raw_texel<C, CONTIG>(t, is.c, in);
    }
}

typedef float f32x3b __attribute__((ext_vector_type(3)));
__device__ f32x3b llvm_raw_buffer_load_v3f32(__amdgpu_buffer_rsrc_t rsrc, int voffset, int soffset,
                                             int aux) __asm("llvm.amdgcn.raw.ptr.buffer.load.v3f32");

// sweep_fill_load_raw through a buffer resource over one source image (r: its span, < 2 GiB):
// texels outside the image read the out-of-range offset, whose loads return 0 -- the same values,
// with no per-texel mask held until the data arrives.
template <int C, int NT, bool CONTIG, int CAP = kSLCap>
__device__ __forceinline__ void sweep_fill_load_rsrc(f32x4 (&stg)[CAP / NT], __amdgpu_buffer_rsrc_t r,
                                                     const ImgStrides& is, int Hs, int Ws, const SweepBox& bx) {
    constexpr int kFill = CAP / NT;
    const int nfp = bx.rows * bx.pitch;
    const float rp = 1.0f / (float)bx.pitch;
    const int sy = (int)is.y * 4, sx = (int)is.x * 4, sc = (int)is.c * 4;
#pragma unroll
    for (int k = 0; k < kFill; ++k) {
        const int idx = threadIdx.x + NT * k;
        int row = (int)((float)idx * rp);  // idx < 2^12: off by at most one, corrected
        row -= row * bx.pitch > idx ? 1 : 0;
        row += (row + 1) * bx.pitch <= idx ? 1 : 0;
        const int x = bx.xl + idx - row * bx.pitch, y = bx.yl + row;
        const bool in = idx < nfp && (unsigned)x < (unsigned)Ws && (unsigned)y < (unsigned)Hs;
        const int off = in ? y * sy + x * sx : kOOB;
        f32x4 v = {0.f, 0.f, 0.f, 0.f};
        if (CONTIG && C == 4) {
            v = llvm_raw_buffer_load_v4f32(r, off, 0, 0);
        } else if (CONTIG && C == 3) {
            const f32x3b q = llvm_raw_buffer_load_v3f32(r, off, 0, 0);
            v[0] = q[0];
            v[1] = q[1];
            v[2] = q[2];
        } else {
#pragma unroll
            for (int c = 0; c < C; ++c) v[c] = llvm_raw_buffer_load_f32(r, off, c * sc, 0);
        }
        stg[k] = v;
    }
}

template <int NT, int CAP = kSLCap>
__device__ __forceinline__ void sweep_fill_store(float4* __restrict__ s_src, const f32x4 (&stg)[CAP / NT]) {
#pragma unroll
    for (int k = 0; k < CAP / NT; ++k) *reinterpret_cast<f32x4*>(&s_src[threadIdx.x + NT * k]) = stg[k];
}

template <int C, int NT, bool CONTIG, int CAP = kSLCap>
__device__ __forceinline__ void sweep_fill_box_raw(float4* __restrict__ s_src, const float* __restrict__ img,
                                                   const ImgStrides& is, int Hs, int Ws, const SweepBox& bx) {
    f32x4 stg[CAP / NT];
    sweep_fill_load_raw<C, NT, CONTIG, CAP>(stg, img, is, Hs, Ws, bx);
    sweep_fill_store<NT, CAP>(s_src, stg);
}

// issue_taps_padded + blend_taps on a RAW source: the same weights and fma chain, taps outside
// the image (NaN coordinates included: med3 maps them to a bound) read as zero
template <int C>
__device__ __forceinline__ f32x4 raw_sample(const float* __restrict__ img, const ImgStrides& is, int Ws, int Hs,
                                            float px, float py) {
    TapSet t;
    const float fx0 = floorf(px), fy0 = floorf(py);
    const float wx = px - fx0, ex = 1.0f - wx;
    const float wy = py - fy0, sy = 1.0f - wy;
    t.nw = sy * ex;
    t.ne = sy * wx;
    t.sw = wy * ex;
    t.se = wy * wx;
    const int cx = (int)__builtin_amdgcn_fmed3f(fx0, -2.0f, (float)Ws);
    const int cy = (int)__builtin_amdgcn_fmed3f(fy0, -2.0f, (float)Hs);
    auto tap = [&](int x, int y) {
        const bool in = (unsigned)x < (unsigned)Ws && (unsigned)y < (unsigned)Hs;
        const float* q = img + (in ? (int64_t)y * is.y + (int64_t)x * is.x : 0);
        return is.c == 1 ? raw_texel<C, true>(q, 1, in) : raw_texel<C, false>(q, is.c, in);
    };
    t.a = tap(cx, cy);
    t.b = tap(cx + 1, cy);
    t.c = tap(cx, cy + 1);
    t.d = tap(cx + 1, cy + 1);
    return blend_taps(t);
}

// A source image read through a buffer resource (plane_sweep_pf_kernel: span < 2 GiB): 32-bit byte
// offsets, and texels outside the image read the out-of-range offset (0) instead of a masked load.
struct RsrcImg {
    __amdgpu_buffer_rsrc_t r;
    int sy4, sx4, sc4;  // byte strides of a row, a pixel, a channel
};

// raw_sample's weights, taps and blend (issue_taps_padded + blend_taps) on a RsrcImg: the same bits
template <int C>
__device__ __forceinline__ f32x4 rsrc_sample(const RsrcImg& ri, int Ws, int Hs, float px, float py) {
    TapSet t;
    const float fx0 = floorf(px), fy0 = floorf(py);
    const float wx = px - fx0, ex = 1.0f - wx;
    const float wy = py - fy0, sy = 1.0f - wy;
    t.nw = sy * ex;
    t.ne = sy * wx;
    t.sw = wy * ex;
    t.se = wy * wx;
    const int cx = (int)__builtin_amdgcn_fmed3f(fx0, -2.0f, (float)Ws);
    const int cy = (int)__builtin_amdgcn_fmed3f(fy0, -2.0f, (float)Hs);
    auto tap = [&](int x, int y) {
        const bool in = (unsigned)x < (unsigned)Ws && (unsigned)y < (unsigned)Hs;
        const int off = in ? y * ri.sy4 + x * ri.sx4 : kOOB;
        f32x4 v = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int c = 0; c < C; ++c) v[c] = llvm_raw_buffer_load_f32(ri.r, off, c * ri.sc4, 0);
        return v;
    };
    t.a = tap(cx, cy);
    t.b = tap(cx + 1, cy);
    t.c = tap(cx, cy + 1);
    t.d = tap(cx + 1, cy + 1);
    return blend_taps(t);
}

// Channel-planar staging (round 5, sweep_soa): the box as C planes of CAP floats instead of CAP
// float4 texels.  A depth-per-lane wave's 16-lane LDS phase reads 16 samples along one epipolar
// line (~1.4 px apart at config 3's widest baseline): as 16-B texels they fall on 16 four-bank
// groups by column mod 16, and columns 16 apart collide (PMC r05, config 3: bank-conflict cycles
// 3.6x the LDS instruction cycles); as 4-B words the columns spread over all 64 banks.  The NW / NE
// (SW / SE) taps of one channel are adjacent words: one ds_read2_b32.  Same values, same blend.
template <int C, int NT, int CAP>
__device__ __forceinline__ void sweep_fill_store_soa(float* __restrict__ s, const f32x4 (&stg)[CAP / NT]) {
#pragma unroll
    for (int k = 0; k < CAP / NT; ++k)
#pragma unroll
        for (int c = 0; c < C; ++c) s[c * CAP + threadIdx.x + NT * k] = stg[k][c];
}

// lds_issue on the channel-planar box: the same origin test and taps (channels >= C read as 0)
template <int C, int CAP>
__device__ __forceinline__ bool lds_issue_soa(const float* __restrict__ tex, const LdsBox& b, float px, float py,
                                              TapSet& t) {
    const float fx0 = floorf(px), fy0 = floorf(py);
    const float wx = px - fx0, ex = 1.0f - wx;
    const float wy = py - fy0, sy = 1.0f - wy;
    t.nw = sy * ex;
    t.ne = sy * wx;
    t.sw = wy * ex;
    t.se = wy * wx;
    const float rx = fx0 - b.xl, ry = fy0 - b.yl;  // exact wherever the origin can be staged
    const float ix = __builtin_amdgcn_fmed3f(rx, 0.0f, b.xspan);
    const float iy = __builtin_amdgcn_fmed3f(ry, 0.0f, b.yspan);
    const float* st = tex + (int)__builtin_fmaf(iy, (float)b.pitch, ix);  // < rows * pitch: exact
    t.a = t.b = t.c = t.d = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int c = 0; c < C; ++c) {
        t.a[c] = st[c * CAP];
        t.b[c] = st[c * CAP + 1];
        t.c[c] = st[c * CAP + b.pitch];
        t.d[c] = st[c * CAP + b.pitch + 1];
    }
    return (__builtin_amdgcn_fmed3f(rx, b.gxl, b.gxh) == rx) & (__builtin_amdgcn_fmed3f(ry, b.gyl, b.gyh) == ry);
}

#ifndef MPIV_SW_NOSAMPLE  // timing probes of the depth-per-lane sweep (wrong volumes; never in a product build)
#define MPIV_SW_NOSAMPLE 0
#endif
#ifndef MPIV_SW_NOSTORE
#define MPIV_SW_NOSTORE 0
#endif
#ifndef MPIV_SW_WAVEBOX
#define MPIV_SW_WAVEBOX 0
#endif
#ifndef MPIV_SW_NOFILL
#define MPIV_SW_NOFILL 0
#endif
// The samples and stores of one staged tile (box bx staged in s_src when bx.pitch > 0), shared by
// plane_sweep_dlane_kernel and plane_sweep_pf_kernel: the same arithmetic, so their volumes are
// bit-identical.
template <int C, bool RAW, int PIX, bool RS = false, bool SOA = false, int CAP = kSLCap>
__device__ __forceinline__ void dlane_tile(const float4* __restrict__ s_src, const SweepBox& bx,
                                           __amdgpu_buffer_rsrc_t r, const PadGeom& pg, const float* __restrict__ imb,
                                           const ImgStrides& is, const SweepParams& sp, float rc_hs, float rc_ws,
                                           const float* __restrict__ k9, const float* __restrict__ m,
                                           const float* __restrict__ depths, float* __restrict__ out,
                                           int64_t out_bstride, int64_t out_pstride, int vec, int b, int x0, int y0,
                                           int np, int nr, int lane, int wave, const RsrcImg* ri = nullptr) {
    const int pitch = bx.pitch;
    const bool all_fast = bx.fast != 0;
    const LdsBox lbx = make_lds_box(bx.xl, bx.yl, bx.rows, pitch, sp.Ws, sp.Hs);
    // Lane -> (pixel of the wave's group, depth).  D <= 64: a group is ppw = 64 / D consecutive
    // pixels and lane l takes pixel l / D, depth l % D (lanes past ppw * D idle), so the group's
    // ppw * D * C floats are one contiguous run of the dense volume.  D > 64: a group is one
    // pixel and the depths go in chunks of 64 (the last one partial).
    const int D = sp.D;
    const int ppw = D <= kWave ? kWave / D : 1;
    const int lp = D <= kWave ? lane / D : 0;             // the lane's pixel within its group
    const int ld = D <= kWave ? lane - lp * D : lane;     // the lane's depth within its chunk
    const int nchunk = (D + kWave - 1) / kWave;
    const int ngroup = (np + ppw - 1) / ppw;              // pixel groups per tile row
    typedef float f32xC __attribute__((ext_vector_type(C), aligned(4)));
    // (tile row, depth chunk, pair of pixel groups) loops, wave-uniform and free of integer
    // divisions (the scalar unit is shared by the CU's waves: per-item divisions measured 3x
    // the SALU instructions)
    for (int tr = 0; tr < nr; ++tr)
    for (int ch = 0; ch < nchunk; ++ch) {
    const int dl = ch * kWave + ld;
    const bool dlive = (D <= kWave ? lane < ppw * D : dl < D);
    const float dq = depths[min(dl, D - 1)];
    float* orow = out + (int64_t)b * out_bstride + ((int64_t)(y0 + tr) * sp.Wt + x0) * out_pstride + (int64_t)dl * C;
    for (int g0 = wave * PIX; g0 < ngroup; g0 += kDLWaves * PIX) {
        float px[PIX], py[PIX], rxs[PIX], rys[PIX], rzs[PIX], dep[PIX];
        float* o[PIX];
        bool live[PIX];
#pragma unroll
        for (int j = 0; j < PIX; ++j) {
            const int pix = (g0 + j) * ppw + lp;
            live[j] = dlive && g0 + j < ngroup && pix < np;
            const int pl = min(pix, np - 1);  // idle lanes recompute the last pixel (not stored)
            ray(k9, (float)(x0 + pl), (float)(y0 + tr), rxs[j], rys[j], rzs[j]);  // pixel2cam_torch, utils.py:370
            dep[j] = dq;
            o[j] = orow + (int64_t)pl * out_pstride;
        }
        float su[PIX], sv[PIX];
        bool fast = true;
#pragma unroll
        for (int j = 0; j < PIX; ++j) {
            const float X = rxs[j] * dep[j], Y = rys[j] * dep[j], Z = rzs[j] * dep[j];
            const float pu = __builtin_fmaf(m[2], Z, __builtin_fmaf(m[1], Y, m[0] * X)) + m[3];
            const float pv = __builtin_fmaf(m[6], Z, __builtin_fmaf(m[5], Y, m[4] * X)) + m[7];
            const float den = __builtin_fmaf(m[10], Z, __builtin_fmaf(m[9], Y, m[8] * X)) + m[11] + 1e-10f;
            if (!all_fast) fast = fast && div2_safe(pu, pv, den);
            div2_fast(pu, pv, den, su[j], sv[j]);  // cam2pixel_torch, utils.py:388-391
        }
        if (__builtin_amdgcn_ballot_w64(!fast)) {  // rare: a quotient outside the fast path's range
#pragma unroll
            for (int j = 0; j < PIX; ++j) {
                const float X = rxs[j] * dep[j], Y = rys[j] * dep[j], Z = rzs[j] * dep[j];
                const float pu = __builtin_fmaf(m[2], Z, __builtin_fmaf(m[1], Y, m[0] * X)) + m[3];
                const float pv = __builtin_fmaf(m[6], Z, __builtin_fmaf(m[5], Y, m[4] * X)) + m[7];
                const float den = __builtin_fmaf(m[10], Z, __builtin_fmaf(m[9], Y, m[8] * X)) + m[11] + 1e-10f;
                if (!div2_safe(pu, pv, den)) {
                    su[j] = div_rn(pu, den);
                    sv[j] = div_rn(pv, den);
                }
            }
        }
#pragma unroll
        for (int j = 0; j < PIX; ++j) {
            const float cx = div_const(su[j] + 0.5f, sp.fhs, rc_hs);  // SWAPPED: x / H, utils.py:444
            const float cy = div_const(sv[j] + 0.5f, sp.fws, rc_ws);  //          y / W
            px[j] = unnormalize(to_grid(cx), sp.half_ws);
            py[j] = unnormalize(to_grid(cy), sp.half_hs);
        }
        f32x4 s[PIX];
        bool staged = pitch > 0 && !MPIV_SW_NOSAMPLE;
        if (MPIV_SW_NOSAMPLE) {  // timing probe: no samples, the stores write the positions
#pragma unroll
            for (int j = 0; j < PIX; ++j) s[j] = f32x4{px[j], py[j], 0.0f, 0.0f};
        }
        if (staged) {  // 16-B tap reads (ds_read_b128: 4 LDS cycles, ds_read_b96 8)
            TapSet ts[PIX];
#pragma unroll
            for (int j = 0; j < PIX; ++j)
                staged = (SOA ? lds_issue_soa<C, CAP>(reinterpret_cast<const float*>(s_src), lbx, px[j], py[j], ts[j])
                              : lds_issue(s_src, lbx, px[j], py[j], ts[j])) &&
                         staged;
#pragma unroll
            for (int j = 0; j < PIX; ++j) s[j] = blend_taps(ts[j]);
            // the unused channels' registers stay allocated until the reads are consumed
            // (else a WAW wait serialises the reads)
#pragma unroll
            for (int j = 0; j < PIX; ++j)
                asm volatile("" ::"v"(ts[j].a), "v"(ts[j].b), "v"(ts[j].c), "v"(ts[j].d));
        }
        if (!MPIV_SW_NOSAMPLE && __builtin_amdgcn_ballot_w64(!staged)) {  // wave-uniform test, then per lane
            if (!staged) {                            // a tap origin not staged: gather from global memory
#pragma unroll
                for (int j = 0; j < PIX; ++j) {
                    if (RS) {
                        s[j] = rsrc_sample<C>(*ri, sp.Ws, sp.Hs, px[j], py[j]);
                    } else if (RAW) {
                        s[j] = raw_sample<C>(imb, is, sp.Ws, sp.Hs, px[j], py[j]);
                    } else {
                        TapSet ts;
                        issue_taps_padded(r, sp.Ws, sp.Hs, pg.Wp, pg.org, pg.row, px[j], py[j], ts);
                        s[j] = blend_taps(ts);
                    }
                    asm volatile("" ::: "memory");
                }
            }
        }
#pragma unroll
        for (int j = 0; j < PIX; ++j) {
            if (live[j] && (!MPIV_SW_NOSTORE || s[j][0] == -12345.0f)) {  // (probe: stores kept only nominally)
                f32xC v;
#pragma unroll
                for (int c = 0; c < C; ++c) v[c] = s[j][c];
                if (vec && MPIV_SWNT) __builtin_nontemporal_store(v, reinterpret_cast<f32xC*>(o[j]));
                else if (vec) *reinterpret_cast<f32xC*>(o[j]) = v;
                else {
#pragma unroll
                    for (int c = 0; c < C; ++c) o[j][c] = v[c];
                }
            }
        }
    }
    }
}

// RAW: the source is the caller's strided tensor (img, is) instead of padded texels (img4, pg).
// SLR target rows per tile, CAP staged texels: (4, 3072) by default; few depths take taller
// tiles (more samples per staged box, abi.hip sweep_tile_rows) with a larger box.
// PIX pixels (samples per lane) per iteration: 1 for few depths (D <= 16), 2 above.
template <int C, bool RAW, int SLR = kSLR, int CAP = kSLCap, int PIX = kDLPix, bool SOA = false>
__global__ __launch_bounds__(kDLThreads) void plane_sweep_dlane_kernel(
    const float4* __restrict__ img4, PadGeom pg, const float* __restrict__ img, ImgStrides is, SweepParams sp,
    float rc_hs, float rc_ws, const float* __restrict__ ki, const float* __restrict__ proj,
    const float* __restrict__ depths, float* __restrict__ out, int64_t out_bstride, int64_t out_pstride, int vec,
    int shrink, int span = 0) {
    static_assert(CAP % kDLThreads == 0, "the box fill writes every staging slot");
    static_assert(!SOA || RAW, "channel-planar staging reads RAW sources");
    __shared__ __attribute__((aligned(16))) float4 s_src[CAP];
    __shared__ SweepBox s_box;

    const int segs = (sp.Wt + kSLP - 1) / kSLP;
    const int b = blockIdx.y;
    const int ty = blockIdx.x / segs;
    const int y0 = ty * SLR, x0 = (blockIdx.x - ty * segs) * kSLP;
    const int np = min(kSLP, sp.Wt - x0), nr = min(SLR, sp.Ht - y0);
    const int lane = threadIdx.x & (kWave - 1), wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const float* k9 = ki + (int64_t)b * 9;
    const float* m = proj + (int64_t)b * 16;
    const __amdgpu_buffer_rsrc_t r =
        make_rsrc(RAW ? nullptr : img4 + (int64_t)b * (pg.plane_bytes / 16), RAW ? 0 : pg.plane_bytes);
    const float* imb = RAW ? img + (int64_t)b * is.b : nullptr;

    SweepBox bx;
    if (MPIV_SW_WAVEBOX) {  // probe: every wave derives the box itself (no barrier before the fill)
        float dmin, dmax, dbad;
        sweep_depth_range(depths, sp.D, lane, dmin, dmax, dbad);
        const SweepBox b0 = sweep_tile_box(k9, m, sp, rc_hs, rc_ws, x0, y0, np, nr, dmin, dmax, dbad, shrink, lane, CAP);
        bx.xl = __builtin_amdgcn_readfirstlane(b0.xl);
        bx.yl = __builtin_amdgcn_readfirstlane(b0.yl);
        bx.rows = __builtin_amdgcn_readfirstlane(b0.rows);
        bx.pitch = __builtin_amdgcn_readfirstlane(b0.pitch);
        bx.fast = __builtin_amdgcn_readfirstlane(b0.fast);
        bx.zero = __builtin_amdgcn_readfirstlane(b0.zero);
    } else {
    if (wave == 0) {
        float dmin, dmax, dbad;
        sweep_depth_range(depths, sp.D, lane, dmin, dmax, dbad);
        const SweepBox bx = sweep_tile_box(k9, m, sp, rc_hs, rc_ws, x0, y0, np, nr, dmin, dmax, dbad, shrink, lane, CAP);
        if (lane == 0) s_box = bx;
    }
    __syncthreads();
    bx.xl = __builtin_amdgcn_readfirstlane(s_box.xl);
    bx.yl = __builtin_amdgcn_readfirstlane(s_box.yl);
    bx.rows = __builtin_amdgcn_readfirstlane(s_box.rows);
    bx.pitch = __builtin_amdgcn_readfirstlane(s_box.pitch);
    bx.fast = __builtin_amdgcn_readfirstlane(s_box.fast);
    bx.zero = __builtin_amdgcn_readfirstlane(s_box.zero);
    }
    if (bx.zero) {  // the tile's output is all +0: store it
        sweep_zero_tile<C, kDLThreads>(out, out_bstride, out_pstride, sp, vec, b, x0, y0, np, nr);
        return;
    }
    if (SOA && bx.pitch > 0) {  // channel-planar staging (RAW sources)
        f32x4 stg[CAP / kDLThreads];
        if (is.c == 1 && C > 1)
            sweep_fill_load_raw<C, kDLThreads, true, CAP>(stg, imb, is, sp.Hs, sp.Ws, bx);
        else
            sweep_fill_load_raw<C, kDLThreads, false, CAP>(stg, imb, is, sp.Hs, sp.Ws, bx);
        sweep_fill_store_soa<C, kDLThreads, CAP>(reinterpret_cast<float*>(s_src), stg);
    } else if (RAW && span > 0 && bx.pitch > 0) {
        // (round 5) the fill through a buffer resource over the source image (span: its bytes, < 2 GiB):
        // texels off the image read the out-of-range offset (0) instead of a masked load -- the same
        // values; D = 10 0.173 vs 0.177 ms, config 3 0.615 vs 0.626 (profiles/r05_sweep_rsfill_ab.jsonl)
        f32x4 stg[CAP / kDLThreads];
        const __amdgpu_buffer_rsrc_t rb = make_rsrc(imb, span);
        if (is.c == 1 && C > 1)
            sweep_fill_load_rsrc<C, kDLThreads, true, CAP>(stg, rb, is, sp.Hs, sp.Ws, bx);
        else
            sweep_fill_load_rsrc<C, kDLThreads, false, CAP>(stg, rb, is, sp.Hs, sp.Ws, bx);
        sweep_fill_store<kDLThreads, CAP>(s_src, stg);
    } else if (bx.pitch > 0 && !MPIV_SW_NOFILL) {
        if (RAW && is.c == 1 && C > 1)
            sweep_fill_box_raw<C, kDLThreads, true, CAP>(s_src, imb, is, sp.Hs, sp.Ws, bx);
        else if (RAW)
            sweep_fill_box_raw<C, kDLThreads, false, CAP>(s_src, imb, is, sp.Hs, sp.Ws, bx);
        else
            sweep_fill_box<kDLThreads, CAP>(s_src, r, pg, bx);
    }
    __syncthreads();

    dlane_tile<C, RAW, PIX, false, SOA, CAP>(s_src, bx, r, pg, imb, is, sp, rc_hs, rc_ws, k9, m, depths, out, out_bstride,
                                             out_pstride, vec, b, x0, y0, np, nr, lane, wave);
}

#if MPIV_AB
// Persistent depth-per-lane sweep with the next tile's box prefetched (round 5).  Per tile,
// plane_sweep_dlane_kernel computes a box, stages it and only then samples: two dependent
// latencies (the box's vertex math, the fill's loads) and two barriers before the first store.
// With few depths that prologue is most of the kernel (PMC r05, 768x1024 sources: ~3350 of the
// 4700 cycles a wave lives at D = 10, and ~3350 of 11900 at D = 64).  Here a block stays
// resident (grid = the blocks that fit at once) and walks the tiles t = lb, lb + G, ... (G
// blocks, XCD-aware: at every step an XCD holds a contiguous run of tiles); while tile t is
// sampled, the source texels of tile t + G are already on their way into registers (issued
// right after t's box was staged; committed to LDS after t's last read), and wave 0 computes
// the box of tile t + 2G after its share of the samples.  The boxes, fills, samples and stores
// are plane_sweep_dlane_kernel's (sweep_tile_box, sweep_fill_load_raw, dlane_tile): the volume
// is bit-identical.  One pixel per lane and iteration (the prefetched fill holds 24 VGPRs).
// Measured SLOWER (A/B build only, sweep_pf=1; profiles/r05_sweep_pf_ab.jsonl): config 3 0.71 vs
// 0.62 ms, D = 10 0.216 vs 0.177 -- the per-tile prologue is already hidden by the 3 blocks per
// CU of the one-tile kernel, and the persistent loop needs 100 VGPRs (4 waves per SIMD) or spills
// at 80.
#ifndef MPIV_PF_NOPF
#define MPIV_PF_NOPF 0  // probe: the next tile's fill issued after this tile's samples
#endif
#ifndef MPIV_PF_WAVES
#define MPIV_PF_WAVES 6  // waves per SIMD the allocator must keep (3 blocks per CU, the LDS limit); 0: free
#endif
template <int C, int PIX>
__global__ __launch_bounds__(kDLThreads) __attribute__((amdgpu_waves_per_eu(MPIV_PF_WAVES > 0 ? MPIV_PF_WAVES : 1)))
void plane_sweep_pf_kernel(
    const float* __restrict__ img, int64_t img_bstride, int sy, int sx, int sc, SweepParams sp, float rc_hs,
    float rc_ws, const float* __restrict__ ki, const float* __restrict__ proj, const float* __restrict__ depths,
    float* __restrict__ out, int64_t out_bstride, int64_t out_pstride, int vec, int shrink, int ntiles, int total,
    int span) {
    constexpr int CAP = kSLCap, SLR = kSLR, kFill = CAP / kDLThreads;
    __shared__ __attribute__((aligned(16))) float4 s_src[CAP];
    __shared__ SweepBox s_box[2];
    const int segs = (sp.Wt + kSLP - 1) / kSLP;
    const int G = gridDim.x;
    const int lb = xcd_logical_block(blockIdx.x, G);
    const int lane = threadIdx.x & (kWave - 1), wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    if (lb >= total) return;  // whole block (the grid is at most `total`); no barrier follows
    struct TileGeo {
        int b, x0, y0, np, nr;
    };
    auto geo = [&](int t) {
        TileGeo q;
        q.b = t / ntiles;
        const int tile = t - q.b * ntiles;
        const int ty = tile / segs;
        q.y0 = ty * SLR;
        q.x0 = (tile - ty * segs) * kSLP;
        q.np = min(kSLP, sp.Wt - q.x0);
        q.nr = min(SLR, sp.Ht - q.y0);
        return q;
    };
    float dmin = 0.0f, dmax = 0.0f, dbad = 0.0f;
    if (wave == 0) sweep_depth_range(depths, sp.D, lane, dmin, dmax, dbad);
    auto box_to = [&](int t, int slot) {  // wave 0
        const TileGeo q = geo(t);
        const SweepBox bx = sweep_tile_box(ki + (int64_t)q.b * 9, proj + (int64_t)q.b * 16, sp, rc_hs, rc_ws, q.x0,
                                           q.y0, q.np, q.nr, dmin, dmax, dbad, shrink, lane, CAP);
        if (lane == 0) s_box[slot] = bx;
    };
    auto read_box = [&](int slot) {
        SweepBox bx;
        bx.xl = __builtin_amdgcn_readfirstlane(s_box[slot].xl);
        bx.yl = __builtin_amdgcn_readfirstlane(s_box[slot].yl);
        bx.rows = __builtin_amdgcn_readfirstlane(s_box[slot].rows);
        bx.pitch = __builtin_amdgcn_readfirstlane(s_box[slot].pitch);
        bx.fast = __builtin_amdgcn_readfirstlane(s_box[slot].fast);
        bx.zero = __builtin_amdgcn_readfirstlane(s_box[slot].zero);
        return bx;
    };
    const ImgStrides is{0, sy, sx, sc};
    f32x4 stg[kFill];
    auto fill_load = [&](const SweepBox& bx, int b) {
        if (bx.zero || bx.pitch == 0) return;  // block-uniform
        const __amdgpu_buffer_rsrc_t rb = make_rsrc(img + (int64_t)b * img_bstride, span);
        if (sc == 1 && C > 1)
            sweep_fill_load_rsrc<C, kDLThreads, true, CAP>(stg, rb, is, sp.Hs, sp.Ws, bx);
        else
            sweep_fill_load_rsrc<C, kDLThreads, false, CAP>(stg, rb, is, sp.Hs, sp.Ws, bx);
    };
    const __amdgpu_buffer_rsrc_t r0 = make_rsrc(nullptr, 0);
    const PadGeom pg0{0, 0, 0, 0};
    int t = lb;
    if (wave == 0) {
        box_to(t, 0);
        if (t + G < total) box_to(t + G, 1);
    }
    __syncthreads();
    SweepBox bx = read_box(0);
    fill_load(bx, t / ntiles);
    for (int i = 0;; ++i) {
        const TileGeo q = geo(t);
        if (!bx.zero && bx.pitch > 0) sweep_fill_store<kDLThreads, CAP>(s_src, stg);
        __syncthreads();  // tile t staged; s_box[(i + 1) & 1] holds tile t + G's box
        const int tn = t + G;
        SweepBox bn;
        if (tn < total) {  // block-uniform: the next tile's texels, in flight while t is sampled
            bn = read_box((i + 1) & 1);
            if (!MPIV_PF_NOPF) fill_load(bn, tn / ntiles);
        }
        if (bx.zero) {
            sweep_zero_tile<C, kDLThreads>(out, out_bstride, out_pstride, sp, vec, q.b, q.x0, q.y0, q.np, q.nr);
        } else {
            // lane-only values re-derived per tile: hoisted out of the tile loop they would stay live
            // across it (the allocator then spills at 6 waves per SIMD)
            const RsrcImg ri{make_rsrc(img + (int64_t)q.b * img_bstride, span), sy * 4, sx * 4, sc * 4};
            dlane_tile<C, true, PIX, true>(s_src, bx, r0, pg0, nullptr, is, sp, rc_hs, rc_ws, ki + (int64_t)q.b * 9,
                                           proj + (int64_t)q.b * 16, depths, out, out_bstride, out_pstride, vec, q.b,
                                           q.x0, q.y0, q.np, q.nr, lane, wave, &ri);
        }
        if (tn >= total) break;  // block-uniform; no barrier follows
        if (MPIV_PF_NOPF) fill_load(bn, tn / ntiles);
        if (wave == 0 && tn + G < total) box_to(tn + G, i & 1);
        __syncthreads();  // every read of tile t's staging is done; s_box[i & 1] holds tile t + 2G's box
        t = tn;
        bx = bn;
    }
}
#endif  // MPIV_AB

// Band-walking depth-per-lane sweep (round 5).  plane_sweep_dlane_kernel stages a fresh box for
// every 4 x 64 tile: its prologue (box from the 8 vertices, fill, two barriers) is paid per tile
// and its fill latency is exposed -- with few depths that prologue is most of the kernel (D = 10:
// 0.28 of HBM).  Here a block walks a BAND of kBandSteps tiles of one 64-pixel column segment,
// top to bottom:
//  * the prologue computes every step's box at once (wave 0: 8 steps x 8 vertices = 64 lanes,
//    sweep_tile_box per 8-lane group) and their union's column range [X0, X0 + bpitch);
//  * source rows live in an LDS RING of NR = cap / bpitch rows of that column range (row y in
//    ring row (y + 2) % NR): a step stages only the rows its box adds below the previous one
//    (~3 of ~12 for config 3), and the next step's rows are loaded into registers while this
//    step is sampled (committed after its end-of-step barrier);
//  * a step whose box does not fit the ring (a jump, a window taller than the ring) reloads its
//    window; a band whose union is too wide, and steps the per-tile kernel would not stage
//    (pitch 0) or would zero, follow the per-tile kernel's rules (the same LdsBox exactness
//    argument: a tap origin read from the ring is one the union box staged).
// The samples, their arithmetic and the stores are plane_sweep_dlane_kernel's: bit-identical.
#if MPIV_AB
constexpr int kBandSteps = 8;                   // 4-row tiles per band (8 x 8 vertices = one wave)
constexpr int kBandFill = 2;                    // prefetched ring texels per thread (1024 per step)

template <int C, int PIX>
__global__ __launch_bounds__(kDLThreads) void plane_sweep_band_kernel(
    const float* __restrict__ img, ImgStrides is, SweepParams sp, float rc_hs, float rc_ws,
    const float* __restrict__ ki, const float* __restrict__ proj, const float* __restrict__ depths,
    float* __restrict__ out, int64_t out_bstride, int64_t out_pstride, int vec, int shrink) {
    constexpr int CAP = kSLCap;
    __shared__ __attribute__((aligned(16))) float4 s_src[CAP];
    __shared__ SweepBox s_box[kBandSteps];
    const int segs = (sp.Wt + kSLP - 1) / kSLP;
    const int b = blockIdx.y;
    const int band = blockIdx.x / segs;
    const int x0 = (blockIdx.x - band * segs) * kSLP;
    const int by0 = band * kSLR * kBandSteps;
    const int np = min(kSLP, sp.Wt - x0);
    const int nsteps = min(kBandSteps, (sp.Ht - by0 + kSLR - 1) / kSLR);
    const int lane = threadIdx.x & (kWave - 1), wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const float* k9 = ki + (int64_t)b * 9;
    const float* m = proj + (int64_t)b * 16;
    const float* imb = img + (int64_t)b * is.b;
    const bool contig = is.c == 1 && C > 1;

    if (wave == 0) {  // every step's box: lanes 8s .. 8s+7 are step s's vertices
        float dmin, dmax, dbad;
        sweep_depth_range(depths, sp.D, lane, dmin, dmax, dbad);
        const int st = min(lane >> 3, nsteps - 1);
        const int y0 = by0 + st * kSLR, nr = min(kSLR, sp.Ht - y0);
        const SweepBox bx = sweep_tile_box(k9, m, sp, rc_hs, rc_ws, x0, y0, np, nr, dmin, dmax, dbad, shrink, lane, CAP);
        if ((lane & 7) == 0 && (lane >> 3) < nsteps) s_box[lane >> 3] = bx;
    }
    __syncthreads();
    // the union of the staged steps' column ranges (block-uniform)
    int X0 = 1 << 30, X1 = -(1 << 30), wmax = 0;
    for (int st = 0; st < nsteps; ++st) {
        const SweepBox& bx = s_box[st];
        if (bx.pitch > 0 && !bx.zero) {
            X0 = min(X0, bx.xl);
            X1 = max(X1, bx.xl + bx.pitch - 1);
            wmax = max(wmax, bx.rows);
        }
    }
    X0 = __builtin_amdgcn_readfirstlane(X0);
    X1 = __builtin_amdgcn_readfirstlane(X1);
    wmax = __builtin_amdgcn_readfirstlane(wmax);
    const int bpitch = X1 >= X0 ? X1 - X0 + 1 : 0;
    const int NR = bpitch > 0 ? CAP / bpitch : 0;
    // ring mode: every staged window fits the ring with room for the next step's new rows
    const bool ring = bpitch > 0 && NR >= wmax + kSLR + 3;
    const float rpitch = bpitch > 0 ? 1.0f / (float)bpitch : 0.0f;

    // one source texel (x, y) of the union's column range as staged (zero outside the image)
    auto texel = [&](int x, int y) -> f32x4 {
        const bool in = (unsigned)x < (unsigned)sp.Ws && (unsigned)y < (unsigned)sp.Hs;
        const float* t = imb + (in ? (int64_t)y * is.y + (int64_t)x * is.x : 0);
        return contig ? raw_texel<C, true>(t, 1, in) : raw_texel<C, false>(t, is.c, in);
    };
    // ring rows [a, a + n): texel idx -> (row, col); returns the count of texels
    auto ring_idx = [&](int idx, int a, int& rr, int& x, int& y) {
        int row = (int)((float)idx * rpitch);  // idx < 2^13: off by at most one, corrected
        row -= row * bpitch > idx ? 1 : 0;
        row += (row + 1) * bpitch <= idx ? 1 : 0;
        const int col = idx - row * bpitch;
        y = a + row;
        x = X0 + col;
        int r = (y + 2) % NR;
        rr = r * bpitch + col;
    };
    f32x4 pre[kBandFill];
    int pre_a = 0, pre_n = 0;  // rows [pre_a, pre_a + pre_n) are in flight in pre
    auto issue_rows = [&](int a, int n) {  // n * bpitch <= kBandFill * kDLThreads
        pre_a = a;
        pre_n = n;
#pragma unroll
        for (int k = 0; k < kBandFill; ++k) {
            const int idx = (int)threadIdx.x + kDLThreads * k;
            int rr, x, y;
            ring_idx(idx, a, rr, x, y);
            pre[k] = idx < n * bpitch ? texel(x, y) : f32x4{0.f, 0.f, 0.f, 0.f};
        }
    };
    auto commit_rows = [&]() {
#pragma unroll
        for (int k = 0; k < kBandFill; ++k) {
            const int idx = (int)threadIdx.x + kDLThreads * k;
            int rr, x, y;
            ring_idx(idx, pre_a, rr, x, y);
            if (idx < pre_n * bpitch) *reinterpret_cast<f32x4*>(&s_src[rr]) = pre[k];
        }
    };
    auto load_rows_now = [&](int a, int n) {  // synchronous, any count (a window reload)
        for (int idx = threadIdx.x; idx < n * bpitch; idx += kDLThreads) {
            int rr, x, y;
            ring_idx(idx, a, rr, x, y);
            *reinterpret_cast<f32x4*>(&s_src[rr]) = texel(x, y);
        }
    };
    // rows a step needs beyond those staged: (hi, bx.yl + rows - 1], or a reload
    int have_lo = 0, have_hi = -(1 << 30);
    auto plan = [&](const SweepBox& bx, int& a, int& n, bool& reload) {
        const int lo = bx.yl, hi = bx.yl + bx.rows - 1;
        reload = !(lo >= have_lo && lo <= have_hi + 1);
        a = reload ? lo : have_hi + 1;
        n = hi - a + 1;
        if (n < 0) n = 0;
    };

    const int D = sp.D;
    const int ppw = D <= kWave ? kWave / D : 1;
    const int lp = D <= kWave ? lane / D : 0;
    const int ld = D <= kWave ? lane - lp * D : lane;
    const int nchunk = (D + kWave - 1) / kWave;
    const int ngroup = (np + ppw - 1) / ppw;
    typedef float f32xC __attribute__((ext_vector_type(C), aligned(4)));

    // the first step's window, and the second's new rows in flight
    if (ring) {
        const SweepBox& b0 = s_box[0];
        if (b0.pitch > 0 && !b0.zero) {
            load_rows_now(b0.yl, b0.rows);
            have_lo = b0.yl;
            have_hi = b0.yl + b0.rows - 1;
        }
    }
    for (int st = 0; st < nsteps; ++st) {
        SweepBox bx;
        bx.xl = __builtin_amdgcn_readfirstlane(s_box[st].xl);
        bx.yl = __builtin_amdgcn_readfirstlane(s_box[st].yl);
        bx.rows = __builtin_amdgcn_readfirstlane(s_box[st].rows);
        bx.pitch = __builtin_amdgcn_readfirstlane(s_box[st].pitch);
        bx.fast = __builtin_amdgcn_readfirstlane(s_box[st].fast);
        bx.zero = __builtin_amdgcn_readfirstlane(s_box[st].zero);
        const int y0 = by0 + st * kSLR, nr = min(kSLR, sp.Ht - y0);
        const bool staged_step = bx.pitch > 0 && !bx.zero;
        if (!ring && staged_step) {  // the per-tile kernel's own box for this step (linear LDS)
            if (contig)
                sweep_fill_box_raw<C, kDLThreads, true, CAP>(s_src, imb, is, sp.Hs, sp.Ws, bx);
            else
                sweep_fill_box_raw<C, kDLThreads, false, CAP>(s_src, imb, is, sp.Hs, sp.Ws, bx);
        }
        if (ring && staged_step && st > 0) {
            int a, n;
            bool reload;
            plan(bx, a, n, reload);
            if (!reload && pre_n > 0 && pre_a == a && pre_n >= n) {
                commit_rows();  // prefetched during the previous step
            } else if (n > 0) {
                load_rows_now(a, n);
            }
            if (reload) have_lo = a;
            have_hi = max(have_hi, a + n - 1);
            have_lo = max(have_lo, have_hi - NR + 1);
        }
        pre_n = 0;
        __syncthreads();  // the step's rows are in LDS
        // the next staged step's new rows: in flight while this step is sampled
        if (ring && st + 1 < nsteps) {
            const SweepBox& bn = s_box[st + 1];
            if (bn.pitch > 0 && !bn.zero) {
                int a, n;
                bool reload;
                plan(bn, a, n, reload);
                // the rows it would overwrite must not be this step's (window + new rows <= NR)
                if (!reload && n > 0 && n * bpitch <= kBandFill * kDLThreads &&
                    (a + n - 1) - (staged_step ? bx.yl : a) + 1 <= NR)
                    issue_rows(a, n);
            }
        }
        if (bx.zero) {
            sweep_zero_tile<C, kDLThreads>(out, out_bstride, out_pstride, sp, vec, b, x0, y0, np, nr);
        } else {
            // this step's box: the ring (rows through the ring map) or the linear per-tile box
            const int pitch = !staged_step ? 0 : ring ? bpitch : bx.pitch;
            const int bxl = ring ? X0 : bx.xl;
            const int sbase = ring ? (bx.yl + 2) % max(NR, 1) : 0;
            const bool all_fast = bx.fast != 0;
            const LdsBox lbx = make_lds_box(bxl, bx.yl, bx.rows, max(pitch, 2), sp.Ws, sp.Hs);
            for (int tr = 0; tr < nr; ++tr)
            for (int ch = 0; ch < nchunk; ++ch) {
            const int dl = ch * kWave + ld;
            const bool dlive = (D <= kWave ? lane < ppw * D : dl < D);
            const float dq = depths[min(dl, D - 1)];
            float* orow = out + (int64_t)b * out_bstride + ((int64_t)(y0 + tr) * sp.Wt + x0) * out_pstride + (int64_t)dl * C;
            for (int g0 = wave * PIX; g0 < ngroup; g0 += kDLWaves * PIX) {
                float px[PIX], py[PIX], rxs[PIX], rys[PIX], rzs[PIX];
                float* o[PIX];
                bool live[PIX];
#pragma unroll
                for (int j = 0; j < PIX; ++j) {
                    const int pix = (g0 + j) * ppw + lp;
                    live[j] = dlive && g0 + j < ngroup && pix < np;
                    const int pl = min(pix, np - 1);
                    ray(k9, (float)(x0 + pl), (float)(y0 + tr), rxs[j], rys[j], rzs[j]);  // pixel2cam_torch, utils.py:370
                    o[j] = orow + (int64_t)pl * out_pstride;
                }
                float su[PIX], sv[PIX];
                bool fast = true;
#pragma unroll
                for (int j = 0; j < PIX; ++j) {
                    const float X = rxs[j] * dq, Y = rys[j] * dq, Z = rzs[j] * dq;
                    const float pu = __builtin_fmaf(m[2], Z, __builtin_fmaf(m[1], Y, m[0] * X)) + m[3];
                    const float pv = __builtin_fmaf(m[6], Z, __builtin_fmaf(m[5], Y, m[4] * X)) + m[7];
                    const float den = __builtin_fmaf(m[10], Z, __builtin_fmaf(m[9], Y, m[8] * X)) + m[11] + 1e-10f;
                    if (!all_fast) fast = fast && div2_safe(pu, pv, den);
                    div2_fast(pu, pv, den, su[j], sv[j]);  // cam2pixel_torch, utils.py:388-391
                }
                if (__builtin_amdgcn_ballot_w64(!fast)) {  // rare: a quotient outside the fast path's range
#pragma unroll
                    for (int j = 0; j < PIX; ++j) {
                        const float X = rxs[j] * dq, Y = rys[j] * dq, Z = rzs[j] * dq;
                        const float pu = __builtin_fmaf(m[2], Z, __builtin_fmaf(m[1], Y, m[0] * X)) + m[3];
                        const float pv = __builtin_fmaf(m[6], Z, __builtin_fmaf(m[5], Y, m[4] * X)) + m[7];
                        const float den = __builtin_fmaf(m[10], Z, __builtin_fmaf(m[9], Y, m[8] * X)) + m[11] + 1e-10f;
                        if (!div2_safe(pu, pv, den)) {
                            su[j] = div_rn(pu, den);
                            sv[j] = div_rn(pv, den);
                        }
                    }
                }
#pragma unroll
                for (int j = 0; j < PIX; ++j) {
                    const float cx = div_const(su[j] + 0.5f, sp.fhs, rc_hs);  // SWAPPED: x / H, utils.py:444
                    const float cy = div_const(sv[j] + 0.5f, sp.fws, rc_ws);  //          y / W
                    px[j] = unnormalize(to_grid(cx), sp.half_ws);
                    py[j] = unnormalize(to_grid(cy), sp.half_hs);
                }
                f32x4 smp[PIX];
                bool staged = pitch > 0;
                if (staged) {
                    TapSet ts[PIX];
#pragma unroll
                    for (int j = 0; j < PIX; ++j) {
                        // lds_issue through the ring's row map (rows r0, r0 + 1 of the ring)
                        TapSet& t = ts[j];
                        const float fx0 = floorf(px[j]), fy0 = floorf(py[j]);
                        const float wx = px[j] - fx0, ex = 1.0f - wx;
                        const float wy = py[j] - fy0, sy = 1.0f - wy;
                        t.nw = sy * ex;
                        t.ne = sy * wx;
                        t.sw = wy * ex;
                        t.se = wy * wx;
                        const float rx = fx0 - lbx.xl, ry = fy0 - lbx.yl;
                        const int ix = (int)__builtin_amdgcn_fmed3f(rx, 0.0f, lbx.xspan);
                        const int iy = (int)__builtin_amdgcn_fmed3f(ry, 0.0f, lbx.yspan);
                        int r0 = iy, r1 = iy + 1;
                        if (ring) {
                            r0 = sbase + iy;
                            r0 -= r0 >= NR ? NR : 0;
                            r1 = r0 + 1 == NR ? 0 : r0 + 1;
                        }
                        const float4* s0 = s_src + r0 * pitch + ix;
                        const float4* s1 = s_src + r1 * pitch + ix;
                        t.a = *reinterpret_cast<const f32x4*>(s0);
                        t.b = *reinterpret_cast<const f32x4*>(s0 + 1);
                        t.c = *reinterpret_cast<const f32x4*>(s1);
                        t.d = *reinterpret_cast<const f32x4*>(s1 + 1);
                        staged = staged && (__builtin_amdgcn_fmed3f(rx, lbx.gxl, lbx.gxh) == rx) &
                                               (__builtin_amdgcn_fmed3f(ry, lbx.gyl, lbx.gyh) == ry);
                    }
#pragma unroll
                    for (int j = 0; j < PIX; ++j) smp[j] = blend_taps(ts[j]);
#pragma unroll
                    for (int j = 0; j < PIX; ++j)
                        asm volatile("" ::"v"(ts[j].a), "v"(ts[j].b), "v"(ts[j].c), "v"(ts[j].d));
                }
                if (__builtin_amdgcn_ballot_w64(!staged)) {
                    if (!staged) {  // a tap origin not staged: gather from global memory
#pragma unroll
                        for (int j = 0; j < PIX; ++j) {
                            smp[j] = raw_sample<C>(imb, is, sp.Ws, sp.Hs, px[j], py[j]);
                            asm volatile("" ::: "memory");
                        }
                    }
                }
#pragma unroll
                for (int j = 0; j < PIX; ++j) {
                    if (live[j]) {
                        f32xC v;
#pragma unroll
                        for (int c = 0; c < C; ++c) v[c] = smp[j][c];
                        if (vec && MPIV_SWNT) __builtin_nontemporal_store(v, reinterpret_cast<f32xC*>(o[j]));
                        else if (vec) *reinterpret_cast<f32xC*>(o[j]) = v;
                        else {
#pragma unroll
                            for (int c = 0; c < C; ++c) o[j][c] = v[c];
                        }
                    }
                }
            }
            }
        }
        __syncthreads();  // every sample of this step has read its rows
    }
}

#endif  // MPIV_AB

// Direct depth-per-lane sweep for few depths (D <= 2 automatic, 3..8 go to the pixel-per-lane
// plane_sweep_px_kernel below; abi.hip sweep_raw_into).  The LDS box
// of plane_sweep_dlane_kernel is sized by the depth RANGE, not the depth count, so with few
// depths it serves few samples per staged texel and the block's two serial latencies (box
// prologue, fill) dominate (D = 10: 0.23-0.26 ms for config 3's sources, 0.25-0.28 of HBM).
// Here nothing is staged: a wave takes ppw = 64 / D consecutive pixels x D depths with
// plane_sweep_dlane_kernel's lane mapping (lane = pixel l / D, depth l % D; its ppw * D * C
// results are one contiguous run of the volume) and gathers the four taps of each sample
// straight from the caller's tensor -- for a fixed depth the wave's ppw pixels read
// neighbouring texels, so the gathers hit L1/L2.  A wave walks kDirG pixel groups of its
// row, two samples in flight per lane.  The per-sample arithmetic is the dlane kernel's
// (bit-identical volume).
constexpr int kDirG = 4;        // pixel groups per wave
constexpr int kDirMaxD = 8;     // deepest volume routed past the LDS staging by default (measured:
                                // D = 6 0.15-0.18 ms direct vs 0.19-0.23 staged, pixel per lane
                                // 0.125; D >= 10 the staged kernel wins)
template <int C>
__global__ __launch_bounds__(256) void plane_sweep_direct_kernel(const float* __restrict__ img, ImgStrides is,
                                                                 SweepParams sp, float rc_hs, float rc_ws, float rD,
                                                                 const float* __restrict__ ki,
                                                                 const float* __restrict__ proj,
                                                                 const float* __restrict__ depths,
                                                                 float* __restrict__ out, int64_t out_bstride,
                                                                 int64_t out_pstride, int vec) {
    const int lane = threadIdx.x & (kWave - 1), wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int b = blockIdx.z, y = blockIdx.y;
    const int D = sp.D;
    const int ppw = kWave / D;                            // pixels per group (scalar)
    const int lp = (int)(((float)lane + 0.5f) * rD);      // lane / D (lane < 64, D <= 64: exact)
    const int d = lane - lp * D;                          // the lane's depth
    const bool dlive = lp < ppw;                          // lanes past ppw * D idle
    const int gbase = (blockIdx.x * 4 + wave) * kDirG;    // this wave's first pixel group
    if (gbase * ppw >= sp.Wt) return;                     // whole wave
    const float dq = depths[min(d, D - 1)];
    const float* k9 = ki + (int64_t)b * 9;
    const float* m = proj + (int64_t)b * 16;
    const float* imb = img + (int64_t)b * is.b;
    float* orow = out + (int64_t)b * out_bstride + (int64_t)y * sp.Wt * out_pstride + (int64_t)d * C;
    typedef float f32xC __attribute__((ext_vector_type(C), aligned(4)));
    for (int gi = 0; gi < kDirG; gi += 2) {
        if ((gbase + gi) * ppw >= sp.Wt) break;  // wave-uniform
        float px[2], py[2], su[2], sv[2];
        bool live[2], fast = true;
        int xs[2];
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const int x = (gbase + gi + j) * ppw + lp;
            live[j] = dlive && x < sp.Wt;
            xs[j] = min(x, sp.Wt - 1);  // idle lanes recompute the last pixel (not stored)
            float rx, ry, rz;
            ray(k9, (float)xs[j], (float)y, rx, ry, rz);  // pixel2cam_torch, utils.py:370
            const float X = rx * dq, Y = ry * dq, Z = rz * dq;
            const float pu = __builtin_fmaf(m[2], Z, __builtin_fmaf(m[1], Y, m[0] * X)) + m[3];
            const float pv = __builtin_fmaf(m[6], Z, __builtin_fmaf(m[5], Y, m[4] * X)) + m[7];
            const float den = __builtin_fmaf(m[10], Z, __builtin_fmaf(m[9], Y, m[8] * X)) + m[11] + 1e-10f;
            fast = fast && div2_safe(pu, pv, den);
            div2_fast(pu, pv, den, su[j], sv[j]);  // cam2pixel_torch, utils.py:388-391
        }
        if (__builtin_amdgcn_ballot_w64(!fast)) {  // rare: a quotient outside the fast path's range
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                float rx, ry, rz;
                ray(k9, (float)xs[j], (float)y, rx, ry, rz);
                const float X = rx * dq, Y = ry * dq, Z = rz * dq;
                const float pu = __builtin_fmaf(m[2], Z, __builtin_fmaf(m[1], Y, m[0] * X)) + m[3];
                const float pv = __builtin_fmaf(m[6], Z, __builtin_fmaf(m[5], Y, m[4] * X)) + m[7];
                const float den = __builtin_fmaf(m[10], Z, __builtin_fmaf(m[9], Y, m[8] * X)) + m[11] + 1e-10f;
                if (!div2_safe(pu, pv, den)) {
                    su[j] = div_rn(pu, den);
                    sv[j] = div_rn(pv, den);
                }
            }
        }
        f32x4 s[2];
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const float cx = div_const(su[j] + 0.5f, sp.fhs, rc_hs);  // SWAPPED: x / H, utils.py:444
            const float cy = div_const(sv[j] + 0.5f, sp.fws, rc_ws);  //          y / W
            px[j] = unnormalize(to_grid(cx), sp.half_ws);
            py[j] = unnormalize(to_grid(cy), sp.half_hs);
            s[j] = raw_sample<C>(imb, is, sp.Ws, sp.Hs, px[j], py[j]);
        }
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            if (live[j]) {
                float* o = orow + (int64_t)xs[j] * out_pstride;
                f32xC v;
#pragma unroll
                for (int c = 0; c < C; ++c) v[c] = s[j][c];
                if (vec) __builtin_nontemporal_store(v, reinterpret_cast<f32xC*>(o));
                else {
#pragma unroll
                    for (int c = 0; c < C; ++c) o[c] = v[c];
                }
            }
        }
    }
}

// Pixel-per-lane sweep for few depths (abi.hip sweep_raw_into; automatic for 3 <= D <= 8,
// profiles/r03_sweep_few_depths_ab.txt): a wave takes PW consecutive
// target pixels of one row x 64/PW depths at a time (lane = pixel lane % PW, depth offset
// lane / PW) and walks the D depths, two such steps in flight (four measured slower: the
// VGPRs cost occupancy).  For one depth the PW lanes
// sample neighbouring source texels, so a tap instruction reads 64/PW runs of the source
// instead of the depth-per-lane kernels' one run per depth, and a pixel's ray is formed once
// for all its depths.  The samples go to a wave-private LDS slot [PW][D*C] and leave as the
// wave's contiguous PW*D*C-float run of the volume (16-B stores where aligned); stored straight
// from the lanes instead (each 64-lane store touching 64 pixel runs) the kernel ran 2-5x
// slower.  No block barrier: each wave owns its slot.  The per-sample arithmetic is
// plane_sweep_direct_kernel's (bit-identical volume).
constexpr int kPxMaxDC = 48;  // deepest D*C staged (LDS: 4 waves x 64 x 48 floats = 48 KiB)
template <int C, int PW>
__global__ __launch_bounds__(256) void plane_sweep_px_kernel(const float* __restrict__ img, ImgStrides is,
                                                             SweepParams sp, float rc_hs, float rc_ws, float rDC,
                                                             const float* __restrict__ ki,
                                                             const float* __restrict__ proj,
                                                             const float* __restrict__ depths,
                                                             float* __restrict__ out, int64_t out_bstride,
                                                             int64_t out_pstride, int vec) {
    static_assert(PW == 32 || PW == 64, "a wave is one or two pixel groups");
    constexpr int DS = kWave / PW;  // depths per step
    extern __shared__ __attribute__((aligned(16))) float px_lds[];  // read through f32x4
    const int lane = threadIdx.x & (kWave - 1), wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int b = blockIdx.z, y = blockIdx.y;
    const int x0 = (blockIdx.x * 4 + wave) * PW;
    if (x0 >= sp.Wt) return;  // whole wave; no barrier follows
    const int D = sp.D, DC = D * C;
    float* slot = px_lds + wave * PW * DC;
    const int pl = lane % PW, dsub = lane / PW;
    const int x = min(x0 + pl, sp.Wt - 1);  // lanes past the row recompute its last pixel (not stored)
    const float* k9 = ki + (int64_t)b * 9;
    const float* m = proj + (int64_t)b * 16;
    const float* imb = img + (int64_t)b * is.b;
    float rx, ry, rz;
    ray(k9, (float)x, (float)y, rx, ry, rz);  // pixel2cam_torch, utils.py:370
    for (int d0 = 0; d0 < D; d0 += 2 * DS) {
        float su[2], sv[2], dq[2];
        int dd[2];
        bool fast = true;
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            dd[j] = d0 + j * DS + dsub;
            dq[j] = depths[min(dd[j], D - 1)];  // past the end: the last depth again (not stored)
            const float X = rx * dq[j], Y = ry * dq[j], Z = rz * dq[j];
            const float pu = __builtin_fmaf(m[2], Z, __builtin_fmaf(m[1], Y, m[0] * X)) + m[3];
            const float pv = __builtin_fmaf(m[6], Z, __builtin_fmaf(m[5], Y, m[4] * X)) + m[7];
            const float den = __builtin_fmaf(m[10], Z, __builtin_fmaf(m[9], Y, m[8] * X)) + m[11] + 1e-10f;
            fast = fast && div2_safe(pu, pv, den);
            div2_fast(pu, pv, den, su[j], sv[j]);  // cam2pixel_torch, utils.py:388-391
        }
        if (__builtin_amdgcn_ballot_w64(!fast)) {  // rare: a quotient outside the fast path's range
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                const float X = rx * dq[j], Y = ry * dq[j], Z = rz * dq[j];
                const float pu = __builtin_fmaf(m[2], Z, __builtin_fmaf(m[1], Y, m[0] * X)) + m[3];
                const float pv = __builtin_fmaf(m[6], Z, __builtin_fmaf(m[5], Y, m[4] * X)) + m[7];
                const float den = __builtin_fmaf(m[10], Z, __builtin_fmaf(m[9], Y, m[8] * X)) + m[11] + 1e-10f;
                if (!div2_safe(pu, pv, den)) {
                    su[j] = div_rn(pu, den);
                    sv[j] = div_rn(pv, den);
                }
            }
        }
        f32x4 s[2];
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const float cx = div_const(su[j] + 0.5f, sp.fhs, rc_hs);  // SWAPPED: x / H, utils.py:444
            const float cy = div_const(sv[j] + 0.5f, sp.fws, rc_ws);  //          y / W
            s[j] = raw_sample<C>(imb, is, sp.Ws, sp.Hs, unnormalize(to_grid(cx), sp.half_ws),
                                 unnormalize(to_grid(cy), sp.half_hs));
        }
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            if (dd[j] < D) {
#pragma unroll
                for (int c = 0; c < C; ++c) slot[pl * DC + dd[j] * C + c] = s[j][c];
            }
        }
    }
    // the wave's LDS writes before its reads of other lanes' samples
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const int npx = min(PW, sp.Wt - x0);
    const int n = npx * DC;  // floats of the wave's pixels
    float* ob = out + (int64_t)b * out_bstride + ((int64_t)y * sp.Wt + x0) * out_pstride;
    if (vec && out_pstride == DC && (((uintptr_t)ob) & 15) == 0) {  // one contiguous run
        const int n4 = n >> 2;
        for (int i = lane; i < n4; i += kWave)
            __builtin_nontemporal_store(reinterpret_cast<const f32x4*>(slot)[i], reinterpret_cast<f32x4*>(ob) + i);
        for (int i = (n4 << 2) + lane; i < n; i += kWave) ob[i] = slot[i];
    } else {  // pixel runs of DC floats, out_pstride apart
        for (int i = lane; i < n; i += kWave) {
            int p = (int)(((float)i + 0.5f) * rDC);  // i / DC (i < 64 * kPxMaxDC: exact)
            const int off = i - p * DC;
            ob[(int64_t)p * out_pstride + off] = slot[i];
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
