// synth.hip -- counter-based synthetic MPI generator (BASELINE config 5: a 256-plane
// 4096x2160 MPI is 36.2 GB, so each GPU generates its own plane shard in HBM instead of
// receiving it; SURVEY.md §7 "Config 5 memory", §8d C5).
//
// Texel channel c of plane p at image pixel (x, y) is a pure function of
// (seed, p, y*W + x, c) -- the plane index is GLOBAL, so any plane range generated on
// any rank is bit-identical to the same planes of the whole MPI:
//   h  = mix(seed + 0x9E3779B9 * (p + 1));  h = mix(h ^ (y*W + x));  h = mix(h + 0x85EBCA6B * (c + 1))
//   u  = (h >> 8) * 2^-24                   (exact: U[0,1) on a 2^-24 grid)
//   rgb = 2u - 1 (exact), alpha = u, plane 0 alpha = 1  (SURVEY §8d C2/C4 distribution)
// with mix = the "lowbias32" integer finaliser.  oracle/mpiv_oracle.c restates it
// (oracle_synth_texel) so the oracle can render any row band of the 36 GB MPI
// procedurally without materialising it.
#include "mpiv_common.hpp"

namespace mpiv {

__host__ __device__ __forceinline__ uint32_t synth_mix(uint32_t x) {
    x ^= x >> 16;
    x *= 0x7feb352du;
    x ^= x >> 15;
    x *= 0x846ca68bu;
    x ^= x >> 16;
    return x;
}

__device__ __forceinline__ float synth_unit(uint32_t h) { return (float)(h >> 8) * 0x1p-24f; }

// One packed plane texel per work-item: grid (padded pixels / 256, planes of the range).
// Border texels (the 2-texel zero frame of the packed layout) are written as zeros.
__global__ __launch_bounds__(256) void synth_packed_kernel(uint32_t seed, int H, int W, int p_begin,
                                                           FastDiv wp_div, float4* __restrict__ packed,
                                                           int64_t plane_stride) {
    const int64_t pix = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (pix >= plane_stride) return;
    const int p = p_begin + (int)blockIdx.y;
    const int yp = (int)fast_div((unsigned)pix, wp_div);
    const int y = yp - kPad, x = (int)pix - yp * (int)wp_div.d - kPad;
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    if ((unsigned)y < (unsigned)H && (unsigned)x < (unsigned)W) {
        const uint32_t hp = synth_mix(seed + 0x9E3779B9u * (uint32_t)(p + 1));
        const uint32_t hx = synth_mix(hp ^ (uint32_t)(y * W + x));
        v.x = 2.0f * synth_unit(synth_mix(hx + 0x85EBCA6Bu * 1u)) - 1.0f;
        v.y = 2.0f * synth_unit(synth_mix(hx + 0x85EBCA6Bu * 2u)) - 1.0f;
        v.z = 2.0f * synth_unit(synth_mix(hx + 0x85EBCA6Bu * 3u)) - 1.0f;
        v.w = p == 0 ? 1.0f : synth_unit(synth_mix(hx + 0x85EBCA6Bu * 4u));
    }
    packed[(int64_t)blockIdx.y * plane_stride + pix] = v;
}

// ---------------------------------------------------------------------------
// gather-rate probe (diagnostic, bench.py's texture-path roofline)
// ---------------------------------------------------------------------------
// What bounds the multi-view render is the vector-memory (texture) path that serves its
// 16-B-per-lane tap gathers (TA busy ~0.88, L2 hit 0.99), not HBM.  This
// probe measures that path's ceiling on the running device: every wave issues 16-B
// buffer loads with the render's access shape (64 consecutive 16-B texels = 1 KiB per
// wave instruction) from a 16 KiB window that stays L1/L2-resident, 8 loads in flight;
// the sums keep the loads live.  Bytes moved = blocks * 256 * iters * 8 * 16.
constexpr int kProbeWindow = 16384;

__global__ __launch_bounds__(256) void probe_gather_kernel(const float4* __restrict__ buf, int iters,
                                                           float* __restrict__ sink) {
    const __amdgpu_buffer_rsrc_t r = make_rsrc(buf, kProbeWindow);
    const int lane = threadIdx.x & (kWave - 1);
    const int base = lane * 16;
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    for (int i = 0; i < iters; ++i) {
        f32x4 v[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) v[k] = llvm_raw_buffer_load_v4f32(r, base + ((i + k + (int)threadIdx.x / 64) & 15) * 1024, 0, 0);
#pragma unroll
        for (int k = 0; k < 8; ++k) acc += v[k];
    }
    if (acc[0] + acc[1] + acc[2] + acc[3] == 1234.5f) sink[threadIdx.x & 3] = acc[0];  // never true for a zero window
}

// Phase marker for rocprofv3 traces (mpiv_mark): an empty kernel whose grid size encodes a tag
// (tag x 64 work-items).  tools/parse_prof.py walks the kernel trace in dispatch order and files every
// later libmpiv dispatch under the last marker's tag, so bench.py's legs and sub-legs that launch the
// same kernel with the same grid (the backward chain with and without checkpoints, in plane groups;
// config 3's drop-in and timed launches) are summarised separately.
__global__ __launch_bounds__(64) void mark_kernel() {}

}  // namespace mpiv
