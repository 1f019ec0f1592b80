// render_ring.hip -- fused warp + over-composite (mpi_render_view_torch, utils.py:267-294)
// on the packed layout with every plane's tile footprint streamed into LDS by LDS-DMA
// several planes ahead (mpiv_render_packed, one or few views per launch).
//
// Why: with one view per launch the direct kernel (render.hip) reads each texel from
// HBM about once, but gathers every bilinear tap through the vector-memory path: four
// 64-lane 16-B gathers per plane-pixel kept the texture addresser ~81 % busy (PMC,
// DESIGN.md §8), and only 2 planes per wave are in flight.  Here a block owns a 64 x TY
// output tile; for each plane the box of texels its samples can touch (~66 x (TY+2)) is
// copied into an LDS ring slot by `buffer_load_dwordx4 ... lds` (1 KiB per wave
// instruction, no VGPRs), NS-1 planes ahead of the plane being composited, and the taps
// become ds_read_b128s.  The texture path then moves each footprint texel once (~1.3
// per pixel instead of 4 taps), and NS-1 planes of HBM reads are in flight per block.
//
// Ring protocol (one barrier per plane): at the top of plane p every wave waits for its
// own fills of plane p (s_waitcnt vmcnt(F*(NS-2)): each wave issues exactly F DMA
// instructions per plane, so its younger fills are those of planes p+1 .. p+NS-2), the
// barrier then publishes all waves' fills and retires plane p-1's slot, which the waves
// refill with plane p+NS-1 before compositing plane p.  The DMA is inline asm: hipcc
// cannot tell which LDS bytes a DMA writes and would otherwise drain vmcnt(0) before
// every ds_read (measured).  Lanes past a footprint, and the fills of
// planes past the range or of planes rendered direct, get the buffer's out-of-range
// offset (no memory access; they write zeros into the free slot).
//
// Footprint boxes (prologue, render_lds.hip's argument): the tile's 4 corners are pushed
// through the exact per-pixel recipe; rounded positions are monotone in the exact ones,
// and while w keeps its sign over the tile its image is the convex hull of the corners,
// so every interior sample lies within one texel of the corner box; the box gets that
// margin and is clipped to the packed plane's 2-texel zero border.  A sample whose tap
// origin is not staged anyway (lds_issue's exactness test: NaN, ill-conditioned
// geometry) gathers from global memory, so the result is bit-identical to the direct
// kernel whatever the boxes cover; planes whose box is not finite or does not fit a slot
// render direct.
#include "mpiv_common.hpp"

#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"

namespace mpiv {

constexpr int kRTX = 64;      // tile width: one wave row
constexpr int kRMaxP = 512;   // planes per launch in the box table
constexpr int kRMaxPitch = 256;

// One LDS-DMA fill instruction: 64 lanes x 16 B from the buffer at per-lane byte offsets
// into LDS bytes [lds, lds + 1 KiB).  M0 carries the LDS base; no kernel in this library
// uses M0 otherwise.
__device__ __forceinline__ void ring_dma16(__amdgpu_buffer_rsrc_t r, int voff, unsigned lds) {
    asm volatile("s_mov_b32 m0, %2\n\tbuffer_load_dwordx4 %0, %1, 0 offen lds" ::"v"(voff), "s"(r), "s"(lds)
                 : "memory", "m0");
}

template <int N>
__device__ __forceinline__ void ring_wait_vm() {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// NW waves per block, RPL output rows per lane (tile height TY = NW * RPL), NS ring slots
// of F * NW * 64 texels.
template <bool CT, int NW, int RPL, int NS, int F>
__global__ __launch_bounds__(NW * 64) void render_ring_kernel(const float4* __restrict__ planes, int64_t plane_stride,
                                                          RenderGeom g, int V, int p_begin, int p_end, int back,
                                                          const float* __restrict__ homs,
                                                          float* __restrict__ out) {
    constexpr int kRWaves = NW;
    constexpr int NT = NW * kWave;
    constexpr int TY = kRWaves * RPL;
    constexpr int CAP = F * kRWaves * kWave;  // texels per slot
    __shared__ __attribute__((aligned(16))) float4 s_tex[NS][CAP];
    __shared__ int2 s_box[kRMaxP];  // per plane: (x_lo, y_lo) and (rows, direct) as 16-bit pairs
    __shared__ int s_pitch;

    const int tiles_x = (g.W + kRTX - 1) / kRTX;
    const int lb = xcd_logical_block(blockIdx.x, gridDim.x);
    const int v = lb % V;
    const int tile = lb / V;
    const int tx0 = (tile % tiles_x) * kRTX, ty0 = (tile / tiles_x) * TY;
    const int lane = threadIdx.x & (kWave - 1), wave = threadIdx.x >> 6;
    const float* hv = homs + (int64_t)v * g.P * 9;
    const int np = p_end - p_begin;

    if (threadIdx.x == 0) s_pitch = 0;
    __syncthreads();

    // ---- prologue: per-plane footprint boxes (thread q -> plane q/4, corner q%4) and the
    // tile-level proof of the fast division (render_packed_kernel)
    const int cx1 = min(tx0 + kRTX - 1, g.W - 1), cy1 = min(ty0 + TY - 1, g.H - 1);
    bool ok_div = true;
    for (int q0 = 0; q0 < 4 * np; q0 += NT) {
        const int q = q0 + (int)threadIdx.x;
        const bool live = q < 4 * np;
        const int pl = p_begin + (live ? (q >> 2) : 0);
        const int corner = q & 3;
        const float fx = (float)((corner & 1) ? cx1 : tx0), fy = (float)((corner & 2) ? cy1 : ty0);
        const float* h = hv + (int64_t)pl * 9;
        if (live && corner == 0) ok_div = ok_div && div2_rect_safe(h, (float)tx0, (float)cx1, (float)ty0, (float)cy1);
        float px, py;
        render_pos<true>(h, fx, fy, g, px, py);
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
            const bool ok = pos || neg;
            const int xl = ok ? max((int)xmin - 1, -2) : 0, xh = ok ? min((int)xmax + 2, g.W + 1) : 0;
            const int yl = ok ? max((int)ymin - 1, -2) : 0, yh = ok ? min((int)ymax + 2, g.H + 1) : 0;
            const int width = xh - xl + 1, rows = yh - yl + 1;
            const int direct = (!ok || width < 2 || rows < 2 || width > kRMaxPitch || width * rows > CAP) ? 1 : 0;
            s_box[q >> 2] = make_int2((xl & 0xFFFF) | (yl << 16), rows | (direct << 16));  // |xl|,|yl| < 2^15
            if (!direct) atomicMax(&s_pitch, width);
        }
    }
    const bool proven = __syncthreads_and(ok_div);
    const int pitch = s_pitch;  // common row pitch of the staged boxes

    // this lane's texels of a fill: idx = (f*4 + wave)*64 + lane -> (row, col) of the box,
    // as a texel offset from the box origin in the padded plane
    int rel[F];
#pragma unroll
    for (int f = 0; f < F; ++f) {
        const int idx = (f * kRWaves + wave) * kWave + lane;
        const int row = pitch > 0 ? idx / pitch : 0;
        rel[f] = row * g.Wp + (idx - row * pitch);
    }
    auto box_of = [&](int i) {
        const int2 b = s_box[i];
        return make_int4((int)(short)(b.x & 0xFFFF), b.x >> 16, b.y & 0xFFFF, b.y >> 16);
    };
    const unsigned lds0 = (unsigned)(uintptr_t)&s_tex[0][0] + (unsigned)wave * kWave * 16;
    auto staged = [&](const int4& bx) { return bx.w == 0 && bx.z * pitch <= CAP; };
    // F fills of plane pl (slot pl % NS); every wave issues exactly F instructions
    auto fill = [&](int pl) {
        const bool in = pl < p_end;
        const int4 bx = box_of(in ? pl - p_begin : 0);
        const bool st = in && staged(bx);
        const int nfp = st ? bx.z * pitch : 0;
        const int org = (bx.y + kPad) * g.Wp + bx.x + kPad;  // >= 0: boxes start at -2
        const __amdgpu_buffer_rsrc_t r = make_rsrc(planes + (int64_t)(in ? pl : p_begin) * plane_stride, g.plane_bytes);
        const unsigned slot = lds0 + (unsigned)((pl - p_begin) % NS) * CAP * 16;
#pragma unroll
        for (int f = 0; f < F; ++f) {
            const int idx = (f * kRWaves + wave) * kWave + lane;
            ring_dma16(r, idx < nfp ? (org + rel[f]) * 16 : kOOB,
                       __builtin_amdgcn_readfirstlane(slot + (unsigned)(f * kRWaves * kWave * 16)));
        }
    };

    float cr[RPL], cg[RPL], cb[RPL], tt[RPL];
#pragma unroll
    for (int k = 0; k < RPL; ++k) {
        cr[k] = -0.0f; cg[k] = -0.0f; cb[k] = -0.0f; tt[k] = 1.0f;  // plane 0 replaces (render.hip)
    }
    const bool replace_first = !CT || back;
    const float fx = (float)(tx0 + lane);

#pragma unroll
    for (int k = 0; k < NS - 1; ++k) fill(p_begin + k);
    for (int p = p_begin; p < p_end; ++p) {
        ring_wait_vm<F * (NS - 2)>();
        __syncthreads();
        fill(p + NS - 1);
        const int4 bx = box_of(p - p_begin);
        const bool st = staged(bx);
        const float4* tex = &s_tex[(p - p_begin) % NS][0];
        const LdsBox box = make_lds_box(bx.x, bx.y, st ? bx.z : 2, pitch > 1 ? pitch : 2, g.W, g.H);
        Hom9 h = load_hom(hv + (int64_t)p * 9);
        const bool first = replace_first && p == p_begin;
#pragma unroll
        for (int k = 0; k < RPL; ++k) {
            const float fy = (float)(ty0 + wave + kRWaves * k);
            float px, py;
            if (proven)
                render_pos_fast<false>(h.h, fx, fy, g, px, py);
            else
                render_pos_fast<true>(h.h, fx, fy, g, px, py);
            TapSet ts;
            bool hit = st && lds_issue(tex, box, px, py, ts);
            if (__builtin_amdgcn_ballot_w64(!hit)) {  // wave-uniform: some sample not staged
                TapSet tg;
                issue_taps_padded(make_rsrc(planes + (int64_t)p * plane_stride, g.plane_bytes), g.W, g.H, g.Wp,
                                  g.org, g.row, px, py, tg);
                if (!hit) ts = tg;
            }
            const f32x4 s = blend_taps(ts);
            const float a = first ? 1.0f : s[3];
            const float om = 1.0f - a;
            cr[k] = over(s[0], a, om, cr[k]);
            cg[k] = over(s[1], a, om, cg[k]);
            cb[k] = over(s[2], a, om, cb[k]);
            if (CT) tt[k] = tt[k] * om;
        }
    }
    ring_wait_vm<0>();  // the past-the-end fills land before the block's LDS is released
    const int x = tx0 + lane;
#pragma unroll
    for (int k = 0; k < RPL; ++k) {
        const int y = ty0 + wave + kRWaves * k;
        if (x >= g.W || y >= g.H) continue;
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

}  // namespace mpiv

#pragma clang diagnostic pop
