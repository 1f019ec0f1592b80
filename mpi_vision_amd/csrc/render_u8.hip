// render_u8.hip -- the fused warp + over-composite on an 8-bit RGBA MPI (4-B texels), the
// reference's own test-MPI format (test/rgba_00..09.png; utils.py:324-331 reads images as
// `t.float() / 255.0`).
//
// Packed u8 layout: [P][H+4][W+4] uint32 (RGBA bytes, little-endian: R in bits 0-7), the
// same plane-major order and 2-texel zero border as mpiv_pack_planes, 4 B per texel
// instead of 16: a single view moves a quarter of the HBM bytes.
//
// Bit-exactness: a tap's channel is converted to the reference's float texel RN(u8/255)
// exactly -- v_cvt_f32_ubyte<k> then fma(x, hi, x*lo) with hi = RN(1/255) and lo =
// RN(1/255 - hi), checked for all 256 values (tests/test_u8_gpu.py; same value as the
// IEEE division) -- and the weights, fma chain and over-operator are render.hip's, so
// the frame equals mpi_render_view_torch(u8.float() / 255) bit for bit.  The conversion
// happens when the taps are blended, so a tap in flight costs one VGPR instead of four.
#include "mpiv_common.hpp"

namespace mpiv {

// RN(x / 255) for x in 0..255 (2 VALU after the byte conversion; exhaustively exact)
__device__ __forceinline__ float u8_unit(unsigned x) {
    const float f = (float)x;
    const float hi = __builtin_bit_cast(float, 998277249u);   // RN(1/255)  = 0x3B808081
    const float lo = __builtin_bit_cast(float, 2944335615u);  // RN(1/255 - hi)
    return __builtin_fmaf(f, hi, f * lo);
}

struct TapSetU8 {
    unsigned a, b, c, d;  // NW, NE, SW, SE texels (RGBA bytes; 0 outside the plane)
    float wx, wy;         // fractional offsets; weights formed at blend time
};

// issue_taps_padded for 4-B texels (org / row in bytes of the u8 padded plane)
__device__ __forceinline__ void issue_taps_u8(__amdgpu_buffer_rsrc_t r, int W, int H, int Wp, int org, int row,
                                              float px, float py, TapSetU8& t) {
    const float fx0 = floorf(px), fy0 = floorf(py);
    t.wx = px - fx0;
    t.wy = py - fy0;
    const int cx = (int)__builtin_amdgcn_fmed3f(fx0, -2.0f, (float)W);
    const int cy = (int)__builtin_amdgcn_fmed3f(fy0, -2.0f, (float)H);
    const int off = (__mul24(cy, Wp) + cx) * 4 + org;  // >= 0, < plane bytes
    t.a = __builtin_bit_cast(unsigned, llvm_raw_buffer_load_f32(r, off, 0, 0));
    t.b = __builtin_bit_cast(unsigned, llvm_raw_buffer_load_f32(r, off + 4, 0, 0));
    t.c = __builtin_bit_cast(unsigned, llvm_raw_buffer_load_f32(r, off + row, 0, 0));
    t.d = __builtin_bit_cast(unsigned, llvm_raw_buffer_load_f32(r, off + row + 4, 0, 0));
}

// blend_taps with the same weight products (issue_taps_padded) and fma chain
__device__ __forceinline__ f32x4 blend_taps_u8(const TapSetU8& t) {
    const float ex = 1.0f - t.wx, sy = 1.0f - t.wy;
    const float nw = sy * ex, ne = sy * t.wx, sw = t.wy * ex, se = t.wy * t.wx;
    f32x4 o;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        float acc = u8_unit((t.a >> (8 * k)) & 255u) * nw;
        acc = __builtin_fmaf(u8_unit((t.b >> (8 * k)) & 255u), ne, acc);
        acc = __builtin_fmaf(u8_unit((t.c >> (8 * k)) & 255u), sw, acc);
        acc = __builtin_fmaf(u8_unit((t.d >> (8 * k)) & 255u), se, acc);
        o[k] = acc;
    }
    return o;
}

struct U8Geom {
    int org;          // byte offset of texel (0, 0) in a padded u8 plane
    int row;          // Wp * 4
    int plane_bytes;  // (H+4)*(W+4)*4
};

// render_rows_pixels on u8 texels: rows y0 .. y0+R-1 of column x, planes outermost,
// two samples in flight (R = 2: one-row-per-lane locality; R = 8: vertical halo reuse)
template <bool CT, bool GUARD, int R>
__device__ __forceinline__ void render_u8_pixels(const unsigned* __restrict__ planes, int64_t plane_stride,
                                                 const RenderGeom& g, const U8Geom& ug, int p_begin, int p_end,
                                                 int back, const float* __restrict__ hv, int x, int y0, float* cr,
                                                 float* cg, float* cb, float* tt) {
    static_assert(R % 2 == 0, "R must be even");
    const float fx = (float)x;
    const bool replace_first = !CT || back;
    const int last = p_end - 1;
    auto hom = [&](int p) { return load_hom(hv + (int64_t)(p < last ? p : last) * 9); };
    auto issue = [&](int p, int k, const Hom9& h, TapSetU8& ts) {
        const int q = p < last ? p : last;
        float px, py;
        render_pos_fast<GUARD>(h.h, fx, (float)(y0 + k), g, px, py);
        issue_taps_u8(make_rsrc(planes + (int64_t)q * plane_stride, ug.plane_bytes), g.W, g.H, g.Wp, ug.org, ug.row,
                      px, py, ts);
    };
    auto consume = [&](const TapSetU8& ts, int k, bool first) {
        const f32x4 s = blend_taps_u8(ts);
        const float a = first ? 1.0f : s[3];
        const float om = 1.0f - a;
        cr[k] = over(s[0], a, om, cr[k]);
        cg[k] = over(s[1], a, om, cg[k]);
        cb[k] = over(s[2], a, om, cb[k]);
        if (CT) tt[k] = tt[k] * om;
    };
    TapSetU8 A, B;
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

// The same with vertical tap reuse (render.hip render_rows_vs_pixels on u8 texels): row k's
// north taps are row k-1's south taps (same clamped offset + one padded row: the same memory
// words) -- and so are their CONVERTED values, so a continuing row converts 2 taps instead of
// 4 (the u8 -> RN(u8/255) conversion is most of this kernel's VALU).  North taps are gathered
// only when some lane of the wave does not continue (wave-uniform branch).
#ifndef MPIV_U8PAIR
#define MPIV_U8PAIR 0  // A/B: the ring's rows consumed two per step (their blends interleaved)
#endif
// D > 2: a ring of D rows in flight (row k + D - 1 issued while row k blends, running on into the
// next planes; the plane loop is unrolled by D / R when D > R so ring positions stay static).  At one view the launch has
// 4 waves per SIMD (R = 4), so the loads each wave keeps in flight are what hides HBM latency.
template <bool CT, bool GUARD, int R, int D = 2>
__device__ __forceinline__ void render_u8_vs_pixels(const unsigned* __restrict__ planes, int64_t plane_stride,
                                                    const RenderGeom& g, const U8Geom& ug, int p_begin, int p_end,
                                                    int back, const float* __restrict__ hv, int x, int y0, float* cr,
                                                    float* cg, float* cb, float* tt) {
    static_assert(R % 2 == 0, "R must be even");
    struct RowU8 {
        unsigned a, b, c, d;  // NW, NE (own, when not shared), SW, SE texels
        float wx, wy;
        int off;
        bool sh, own;
    };
    const float fx = (float)x;
    const bool replace_first = !CT || back;
    const int last = p_end - 1;
    auto hom = [&](int p) { return load_hom(hv + (int64_t)(p < last ? p : last) * 9); };
    auto issue = [&](int p, int k, const Hom9& h, int prev_off, bool can_share, RowU8& t) {
        const int q = p < last ? p : last;
        float px, py;
        render_pos_fast<GUARD>(h.h, fx, (float)(y0 + k), g, px, py);
        const float fx0 = floorf(px), fy0 = floorf(py);
        t.wx = px - fx0;
        t.wy = py - fy0;
        const int cx = (int)__builtin_amdgcn_fmed3f(fx0, -2.0f, (float)g.W);
        const int cy = (int)__builtin_amdgcn_fmed3f(fy0, -2.0f, (float)g.H);
        const int off = (__mul24(cy, g.Wp) + cx) * 4 + ug.org;
        t.off = off;
        t.sh = can_share && off == prev_off + ug.row;
        const __amdgpu_buffer_rsrc_t r = make_rsrc(planes + (int64_t)q * plane_stride, ug.plane_bytes);
        t.c = __builtin_bit_cast(unsigned, llvm_raw_buffer_load_f32(r, off + ug.row, 0, 0));
        t.d = __builtin_bit_cast(unsigned, llvm_raw_buffer_load_f32(r, off + ug.row + 4, 0, 0));
        t.own = __builtin_amdgcn_ballot_w64(!t.sh) != 0;
        if (t.own) {  // wave-uniform: some lane needs its own north taps
            t.a = __builtin_bit_cast(unsigned, llvm_raw_buffer_load_f32(r, t.sh ? kOOB : off, 0, 0));
            t.b = __builtin_bit_cast(unsigned, llvm_raw_buffer_load_f32(r, (t.sh ? kOOB - 4 : off) + 4, 0, 0));
        }
    };
    // pc, pd: the previous row's converted south taps; sc, sd: this row's (out)
    auto consume = [&](const RowU8& t, const f32x4& pc, const f32x4& pd, int k, bool first, f32x4& sc,
                       f32x4& sd) {
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            sc[c] = u8_unit((t.c >> (8 * c)) & 255u);
            sd[c] = u8_unit((t.d >> (8 * c)) & 255u);
        }
        f32x4 na = pc, nb = pd;
        if (t.own) {
            asm volatile("");  // a real wave-uniform branch (render.hip MPIV_VS_ASMBR)
#pragma unroll
            for (int c = 0; c < 4; ++c) {
                const float ua = u8_unit((t.a >> (8 * c)) & 255u), ub = u8_unit((t.b >> (8 * c)) & 255u);
                na[c] = t.sh ? pc[c] : ua;
                nb[c] = t.sh ? pd[c] : ub;
            }
        }
        const float ex = 1.0f - t.wx, sy = 1.0f - t.wy;
        const float nw = sy * ex, ne = sy * t.wx, sw = t.wy * ex, se = t.wy * t.wx;
        f32x4 s;
#pragma unroll
        for (int c = 0; c < 4; ++c) {  // blend_taps_u8's fma chain
            float acc = na[c] * nw;
            acc = __builtin_fmaf(nb[c], ne, acc);
            acc = __builtin_fmaf(sc[c], sw, acc);
            acc = __builtin_fmaf(sd[c], se, acc);
            s[c] = acc;
        }
        const float a = first ? 1.0f : s[3];
        const float om = 1.0f - a;
        cr[k] = over(s[0], a, om, cr[k]);
        cg[k] = over(s[1], a, om, cg[k]);
        cb[k] = over(s[2], a, om, cb[k]);
        if (CT) tt[k] = tt[k] * om;
        if (!MPIV_U8PAIR || D == 2) {
            asm volatile("" : "+v"(cr[k]), "+v"(cg[k]), "+v"(cb[k]));  // pinned here (render.hip)
            if (CT) asm volatile("" : "+v"(tt[k]));
        }
    };
    f32x4 pc = {0.f, 0.f, 0.f, 0.f}, pd = pc;
    Hom9 h = hom(p_begin), hn = hom(p_begin + 1);
    if constexpr (D != 2) {
        static_assert((R % D == 0 || D % R == 0) && D > 2, "ring positions must repeat every plane group");
        constexpr int U = D > R ? D / R : 1;       // planes per unrolled group (static ring positions)
        constexpr int NH = (R + D - 2) / R + 1;    // homographies live at once: planes p .. p+NH-1
        RowU8 T[D];
        Hom9 hq[NH];
#pragma unroll
        for (int j = 0; j < NH; ++j) hq[j] = hom(p_begin + j);
        constexpr int KS = MPIV_U8PAIR ? 2 : 1;  // rows consumed per step (A/B: two interleaved blends)
        constexpr int AHEAD = D - KS;             // rows issued ahead of the one consumed
#pragma unroll
        for (int it = 0; it < AHEAD; ++it)
            issue(p_begin + it / R, it % R, hq[it / R], it % R ? T[(it + D - 1) % D].off : 0, it % R != 0, T[it % D]);
        for (int p = p_begin; p < p_end; p += U) {
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int pu = p + u;
                if (U > 1 && pu >= p_end) break;  // wave-uniform: an odd tail plane
                const bool first = replace_first && pu == p_begin;
#pragma unroll
                for (int k0 = 0; k0 < R; k0 += KS) {
#pragma unroll
                    for (int k = k0; k < k0 + KS; ++k) {
                        const int it = u * R + k;  // the row consumed now (item of the group)
                        const int ia = it + AHEAD;  // the row issued now: plane pu + dp (past the end: the last plane again)
                        const int dp = ia / R - u, row = ia % R;
                        issue(pu + dp, row, hq[dp], T[(ia + D - 1) % D].off, row != 0, T[ia % D]);
                    }
                    asm volatile("" ::: "memory");
                    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                    for (int k = k0; k < k0 + KS; ++k) {
                        f32x4 sc, sd;
                        consume(T[(u * R + k) % D], pc, pd, k, first, sc, sd);
                        pc = sc;
                        pd = sd;
                    }
                    if (MPIV_U8PAIR) {
#pragma unroll
                        for (int k = k0; k < k0 + KS; ++k) {
                            asm volatile("" : "+v"(cr[k]), "+v"(cg[k]), "+v"(cb[k]));
                            if (CT) asm volatile("" : "+v"(tt[k]));
                        }
                    }
                }
#pragma unroll
                for (int j = 0; j + 1 < NH; ++j) hq[j] = hq[j + 1];
                hq[NH - 1] = hom(pu + NH);
            }
        }
        return;
    }
    RowU8 A, B;
    issue(p_begin, 0, h, 0, false, A);
    for (int p = p_begin; p < p_end; ++p) {
        const bool first = replace_first && p == p_begin;
#pragma unroll
        for (int k = 0; k < R; k += 2) {  // A holds (p, k)
            issue(p, k + 1, h, A.off, true, B);
            asm volatile("" ::: "memory");
            __builtin_amdgcn_sched_barrier(0);
            f32x4 sc, sd;
            consume(A, pc, pd, k, first, sc, sd);
            pc = sc;
            pd = sd;
            if (k + 2 < R)
                issue(p, k + 2, h, B.off, true, A);
            else
                issue(p + 1, 0, hn, 0, false, A);  // past the end: the last plane again (cached, unused)
            asm volatile("" ::: "memory");
            __builtin_amdgcn_sched_barrier(0);
            consume(B, pc, pd, k + 1, first, sc, sd);
            pc = sc;
            pd = sd;
        }
        h = hn;
        hn = hom(p + 2);
    }
}

// render_rows_kernel's contract on the packed u8 layout (FAST recipe: H, W >= 2): a
// 256-thread block = 64 x 4R tile, XCD-aware (tile, view) order, tile-level division
// proof; a tile where the proof fails runs the per-sample guarded recipe (GUARD).
template <bool CT, int R, bool VS = false, int D = 2>
__global__ __launch_bounds__(256) void render_u8_kernel(const unsigned* __restrict__ planes, int64_t plane_stride,
                                                        RenderGeom g, U8Geom ug, int V, int p_begin, int p_end,
                                                        int back, const float* __restrict__ homs,
                                                        float* __restrict__ out) {
    constexpr int TY = 4 * R;
    const int tiles_x = (g.W + kTileX - 1) / kTileX;
    const int lb = xcd_logical_block(blockIdx.x, gridDim.x);
    const int v = lb % V;
    const int tile = lb / V;
    const int tx0 = (tile % tiles_x) * kTileX, ty0 = (tile / tiles_x) * TY;
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
    if (x >= g.W || y0 >= g.H) return;  // rows past H inside [y0, y0+R) are computed, not stored
    float cr[R], cg[R], cb[R], tt[R];
#pragma unroll
    for (int k = 0; k < R; ++k) {
        cr[k] = -0.0f; cg[k] = -0.0f; cb[k] = -0.0f; tt[k] = 1.0f;  // render_packed_pixel: plane 0 replaces
    }
    if (dead) {  // every plane samples the zero border over the whole tile (render.hip tile_dead)
        composite_zero<CT>(p_begin, p_end, !CT || back, cr[0], cg[0], cb[0], tt[0]);
#pragma unroll
        for (int k = 1; k < R; ++k) {
            cr[k] = cr[0]; cg[k] = cg[0]; cb[k] = cb[0]; tt[k] = tt[0];
        }
    } else if (proven) {
        if constexpr (VS)
            render_u8_vs_pixels<CT, false, R, D>(planes, plane_stride, g, ug, p_begin, p_end, back, hv, x, y0, cr, cg,
                                                 cb, tt);
        else
            render_u8_pixels<CT, false, R>(planes, plane_stride, g, ug, p_begin, p_end, back, hv, x, y0, cr, cg, cb,
                                           tt);
    } else {  // rare (w near 0 over the tile): the guarded recipe two rows at a time (few VGPRs)
#pragma unroll
        for (int k = 0; k < R; k += 2)
            render_u8_pixels<CT, true, 2>(planes, plane_stride, g, ug, p_begin, p_end, back, hv, x, y0 + k, cr + k,
                                          cg + k, cb + k, tt + k);
    }
#pragma unroll
    for (int k = 0; k < R; ++k) {
        const int y = y0 + k;
        if (y >= g.H) break;
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

// [H,W,P,4] uint8 (element strides y, x, p, c) -> packed u8 planes [P][H+4][W+4] uint32,
// zero border.  A block moves 64 padded pixels x 16 planes through LDS (reads: a pixel's
// 16 planes are 64 contiguous bytes; writes: 64 texels = 256 B per plane).
__global__ __launch_bounds__(256) void pack_planes_u8_kernel(const uint8_t* __restrict__ mpi, NativeStrides s, int H,
                                                             int W, int P, FastDiv wp_div, unsigned* __restrict__ packed,
                                                             int64_t plane_stride) {
    __shared__ unsigned tile[kPackPl][kPackPix + 1];
    const int64_t npix = plane_stride;
    const int64_t pix0 = (int64_t)blockIdx.x * kPackPix;
    const int p0 = blockIdx.y * kPackPl;
    for (int k = threadIdx.x; k < kPackPix * kPackPl; k += blockDim.x) {
        const int j = k % kPackPl, i = k / kPackPl;
        const int64_t pix = pix0 + i;
        const int p = p0 + j;
        unsigned val = 0;
        if (pix < npix && p < P) {
            const int yp = (int)fast_div((unsigned)pix, wp_div);
            const int yy = yp - kPad, xx = (int)pix - yp * (int)wp_div.d - kPad;
            if ((unsigned)yy < (unsigned)H && (unsigned)xx < (unsigned)W) {
                const uint8_t* src = mpi + (int64_t)yy * s.y + (int64_t)xx * s.x + (int64_t)p * s.p;
                if (s.c == 1 && ((reinterpret_cast<uintptr_t>(src) & 3) == 0))
                    val = *reinterpret_cast<const unsigned*>(src);
                else
                    val = (unsigned)src[0] | ((unsigned)src[s.c] << 8) | ((unsigned)src[2 * s.c] << 16) |
                          ((unsigned)src[3 * s.c] << 24);
            }
        }
        tile[j][i] = val;
    }
    __syncthreads();
    for (int k = threadIdx.x; k < kPackPix * kPackPl; k += blockDim.x) {
        const int i = k % kPackPix, j = k / kPackPix;
        const int64_t pix = pix0 + i;
        const int p = p0 + j;
        if (pix < npix && p < P) packed[(int64_t)p * plane_stride + pix] = tile[j][i];
    }
}

// Packed u8 planes -> packed float planes (the same padded [P][H+4][W+4] layout as
// mpiv_pack_planes), every channel RN(u8/255) exactly (u8_unit): the texels of the float MPI
// u8.float() / 255 the reference renders.  The many-view route of the u8 render: at 125 views per
// launch the float rows kernel (texture path and VALU co-limited) beats the u8 kernel (VALU-bound
// on the per-tap conversion), so a camera path converts its 8-bit MPI once.
// One texel per work-item: a 4-B read, a 16-B write.
__global__ __launch_bounds__(256) void unpack_u8_planes_kernel(const unsigned* __restrict__ src,
                                                               float4* __restrict__ dst, int64_t n) {
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
        const unsigned t = src[i];
        dst[i] = make_float4(u8_unit(t & 255u), u8_unit((t >> 8) & 255u), u8_unit((t >> 16) & 255u), u8_unit(t >> 24));
    }
}

// Counter-based synthetic u8 MPI (synth.hip's hash; bytes = top 8 bits of each channel's
// hash, plane 0 alpha 255), straight into the packed u8 layout: a config-5 shard per GPU.
__global__ __launch_bounds__(256) void synth_packed_u8_kernel(uint32_t seed, int H, int W, int p_begin,
                                                              FastDiv wp_div, unsigned* __restrict__ packed,
                                                              int64_t plane_stride) {
    const int64_t pix = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (pix >= plane_stride) return;
    const int p = p_begin + (int)blockIdx.y;
    const int yp = (int)fast_div((unsigned)pix, wp_div);
    const int y = yp - kPad, x = (int)pix - yp * (int)wp_div.d - kPad;
    unsigned v = 0;
    if ((unsigned)y < (unsigned)H && (unsigned)x < (unsigned)W) {
        const uint32_t hp = synth_mix(seed + 0x9E3779B9u * (uint32_t)(p + 1));
        const uint32_t hx = synth_mix(hp ^ (uint32_t)(y * W + x));
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            const unsigned byte = (c == 3 && p == 0) ? 255u : (synth_mix(hx + 0x85EBCA6Bu * (uint32_t)(c + 1)) >> 24);
            v |= byte << (8 * c);
        }
    }
    packed[(int64_t)blockIdx.y * plane_stride + pix] = v;
}

}  // namespace mpiv
