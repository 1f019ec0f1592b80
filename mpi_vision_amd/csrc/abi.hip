// abi.hip -- extern "C" entry points of libmpiv.so (declared in include/mpiv.h).
// Unity build: the kernel sources are included here so the library is one
// code object.  Entry points validate shapes/alignment, launch on the caller's
// stream, and report failures through a thread-local message; they never allocate,
// synchronise or abort.
#include <cstdio>
#include <cstdarg>
#include <cstring>
#include <cstdlib>
#include <algorithm>
#include <mutex>

#include "../../include/mpiv.h"

// MPIV_AB=1 (libmpiv_ab.so): also compile the kernel variants kept for A/B measurement
#ifndef MPIV_AB
#define MPIV_AB 0
#endif
#include "render.hip"
#include "render_lds.hip"
#include "render_chunk.hip"
#include "render_ring.hip"
#include "render_mv.hip"
#include "render_bwd.hip"
#include "sweep.hip"
#include "geometry.hip"
#include "assemble.hip"
#include "synth.hip"
#include "render_u8.hip"

namespace {

thread_local char g_err[512] = "";

int fail(int code, const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
    return code;
}

int launched(const char* what) {
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return fail(MPIV_ERR_HIP, "%s: launch failed: %s", what, hipGetErrorString(e));
    g_err[0] = '\0';
    return MPIV_OK;
}

inline hipStream_t S(void* s) { return reinterpret_cast<hipStream_t>(s); }
inline bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }
inline unsigned blocks(int64_t n, int per) { return (unsigned)((n + per - 1) / per); }

// Debug / A/B options (mpiv_debug_set; the defaults are the production dispatch and
// production callers never set them):
//   render_mv=1        launches of >= 4 views use the multi-view LDS kernel (render_mv.hip)
//   render_pair=1|2    the direct render takes pixel pairs sharing taps (render_pair_kernel)
//   render_native_lds=0  mpiv_render gathers directly from the [B,H,W,P,4] tensor
//   render_chunk=-1|4|8|104|108  mpiv_render's in-place chunked kernel off, or CH planes per
//                      chunk (+100: two composite phases per chunk); default 0 = automatic
//                      (8, or 4 for P <= 4)
//   render_ring=-1|0|1..6  packed render through the LDS-DMA ring kernel (render_ring.hip):
//                      off / automatic / forced with geometry k (kRingGeo: waves, rows per
//                      lane, slots, fills per wave and plane)
//   render_tile=-1|0|2|4|8|16|108|116|132  packed render with R rows per work-item
//                      (render_rows_kernel; 100+R: state in LDS, render_rows_lds_kernel);
//                      -1: off (one row per work-item), 0: automatic (R = 8 where it pays)
//   sweep_tile=1       the sweep uses the tile kernel; sweep_store=k (k >= 0) the grouped one
//   render_vshare=-1|0|1  render_rows_kernel without vertical tap reuse (R = render_tile or 8) /
//                      automatic / with it, two rows in flight (R = 8); 3|4|5|11: with it and
//                      (R, rows in flight) = (8, 4) / (6, 3) / (9, 3) / (4, 4)
//   sweep_dlane=0      the LDS sweep runs pixel-per-lane (plane_sweep_lds_kernel) instead of
//                      depth-per-lane (plane_sweep_dlane_kernel)
//   sweep_rows=4|6|8   mpiv_plane_sweep[_into]'s depth-per-lane kernel with tiles of that many
//                      target rows (staging 3072 / 4096 / 4096 texels; 0 = automatic)
//   bwd_gather=0|1|2|3 render backward gather: block tiles (bwd_gather_kernel) / one texel row per
//                      wave, no block barriers (bwd_gather_wave_kernel) / staging and texel waves
//                      (bwd_gather_ws_kernel) / block tiles with the d samples streamed into LDS
//                      one pass ahead (bwd_gather_dma_kernel)
//   chunk_flight=2|4   render_chunk_kernel with that many sub-steps' taps in flight per wave
//                      (0 = automatic)
//   chunk_rows=1|2|4   render_chunk_kernel (mpiv_render / mpiv_render_train) with that many rows per
//                      wave (0 = automatic)
//   bwd_group=k        test hook: the render backward's plane groups of k planes (rounded up to whole
//                      8-plane chunks; the workspace size follows), 0 = automatic (bwd_group_planes)
//   u8_flight=2|4|8    the u8 texel render with vertical reuse: rows in flight per work-item
//                      (0 = automatic: 4 for launches under 2048 blocks)
//   chunk_strip=0|1    the in-place render at CH = 8, one row: render_chunk_kernel's 64 x 1 wave rows
//                      (0) or render_chunk_strip_kernel's 8 x 16 strips with vertical tap reuse (1);
//                      A/B: 2 = 8 x 8 strips, 3 = 8 x 8 with 3 rows in flight, 4 = 8 x 16 with 3,
//                      5 = 8 x 16 with the homographies read through the caches (4 blocks per CU)
//   sweep_direct=-1|0|1  mpiv_plane_sweep[_into] without LDS staging (plane_sweep_direct_kernel):
//                      never / automatic (D <= 2) / for any D <= 64; 2|3: pixel per lane, the wave's
//                      samples staged in LDS (plane_sweep_px_kernel, D * C <= 48; 64 / 32 pixels
//                      per wave; automatic: 64 for 3 <= D <= 8)
//   box_shrink=k       LDS-staged kernels stage boxes k texels narrower per side, which
//                      forces their per-sample global fallback (tests)
//   bwd_fallback=1     mpiv_render_backward skips the tile gather and runs its bucket
//                      fallback for every view (tests)
//   bwd_poll_limit=k   (A/B build) the backward fallback's waits also give up after k polls (the
//                      production limit is 60 s of wall clock per wait); -1: at the first wait -- tests provoke the abort path with it (NaN
//                      gradient, counted by mpiv_render_backward_status)
//   bwd_fb_mode=1|2    (A/B build) the fallback's phases at grid barriers (round 3's schedule,
//                      bwd_fallback_barrier_kernel) / the ticket kernel with a fixed item order (block b:
//                      b, b + nblk, ...; diagnosis)
//   bwd_fb_blocks=k    (A/B build) the backward fallback launches k blocks instead of the resident count
//   netout_geo=WRD     render_netout_kernel<W, R, D>: W waves per block, R rows per work-item
//                      (64 x W*R tiles), D planes' w / a loads in flight (e.g. 821); + 1000: two staged
//                      boxes, one barrier per plane (1821, the default; 0 = automatic)
//   sweep_band=0|1     (A/B build) mpiv_plane_sweep[_into]'s LDS-staged route: one box per 4-row tile
//                      (plane_sweep_dlane_kernel, 0 = default) or bands of 8 tiles with the source rows
//                      in an LDS ring (plane_sweep_band_kernel: measured 15-20 % slower)
//   bwd_overlap=0|1    (A/B build) render backward of views with several plane groups: sequential groups
//                      (0 = default) or the overlapped schedule (group k's gather on a second stream beside
//                      group k-1's chain, two d-sample windows: measured no faster)
//   netout_buf=0|1     render_netout_kernel's staged loads through pointers (0) or buffer resources
//                      with 32-bit offsets (1, default where the spans fit)
//   sweep_pf=0|1       (A/B build) mpiv_plane_sweep[_into]'s LDS-staged route: one block per tile
//                      (plane_sweep_dlane_kernel, 0 = default) or resident blocks walking the tiles with
//                      the next tile's box and texels prefetched (plane_sweep_pf_kernel: measured 15-22 %
//                      slower)
//   sweep_soa=0|1      (A/B build) mpiv_plane_sweep[_into]'s depth-per-lane kernel stages its box as
//                      float4 texels (0 = default) or as channel planes (1: measured 4-7 % slower)
//   render_same=-1|0|1|2  render_rows_kernel's same-row tap reuse (render.hip SAME): off / automatic
//                      (where the sample advances <= 0.8 texel rows per output row; R = 6 then, with
//                      OOB for launches of <= 2 views) / on / on with OOB
//   bwd_margin=k       the tile gather's pixel-window margin in 1/64 pixel (default 16);
//                      negative values make windows miss contributors, which the pair
//                      count must catch (tests)
// Relaxed atomics: a launch reads each option once; setting options while another thread
// launches is a test-harness race on which kernel runs, never on memory.
enum DebugOpt { kOptRenderMv, kOptRenderPair, kOptNativeLds, kOptSweepTile, kOptSweepStore, kOptBoxShrink,
                kOptRenderChunk, kOptRenderRing, kOptRenderTile, kOptBwdFallback, kOptBwdMargin, kOptSweepDlane,
                kOptRenderVshare, kOptChunkRows, kOptSweepRows, kOptChunkFlight, kOptBwdGather, kOptSweepDirect,
                kOptBwdPollLimit, kOptBwdFbBlocks, kOptBwdFbMode, kOptChunkStrip, kOptU8Flight, kOptBwdGroup,
                kOptNetoutGeo, kOptNetoutBuf, kOptBwdOverlap, kOptSweepBand, kOptSweepPf, kOptSweepSoa, kOptBwdUnfold,
                kOptNetoutFg3, kOptRenderSame, kNumOpts };
const char* const kOptNames[kNumOpts] = {"render_mv", "render_pair", "render_native_lds",
                                         "sweep_tile", "sweep_store", "box_shrink", "render_chunk", "render_ring",
                                         "render_tile", "bwd_fallback", "bwd_margin", "sweep_dlane",
                                         "render_vshare", "chunk_rows", "sweep_rows", "chunk_flight", "bwd_gather",
                                         "sweep_direct", "bwd_poll_limit", "bwd_fb_blocks", "bwd_fb_mode",
                                         "chunk_strip", "u8_flight", "bwd_group", "netout_geo", "netout_buf", "bwd_overlap", "sweep_band",
                                         "sweep_pf", "sweep_soa", "bwd_unfold", "netout_fg3",
                                         "render_same"};
#ifndef MPIV_CHUNK_STRIP
#define MPIV_CHUNK_STRIP 1  // round 4: 0.506 vs 0.64 ms in place (profiles/r04j_strip*_ab.jsonl)
#endif
#ifndef MPIV_U8_FLIGHT
#define MPIV_U8_FLIGHT 0
#endif
const int kOptDefaults[kNumOpts] = {0, 0, 1, 0, -1, 0, 0, 0, 0, 0, 16, 1, 0, 0, 0, 0, 0, 0, 0, 0, 0, MPIV_CHUNK_STRIP,
                                    MPIV_U8_FLIGHT, 0, 0, 1, 0, 0, 0, 0, 0, 1, 0};
int g_opts[kNumOpts] = {0, 0, 1, 0, -1, 0, 0, 0, 0, 0, 16, 1, 0, 0, 0, 0, 0, 0, 0, 0, 0, MPIV_CHUNK_STRIP, MPIV_U8_FLIGHT, 0,
                        0, 1, 0, 0, 0, 0, 0, 1, 0};

int opt(DebugOpt o) { return __atomic_load_n(&g_opts[o], __ATOMIC_RELAXED); }

// Option values that select a kernel kept for A/B measurement only: those kernels are
// compiled into libmpiv_ab.so (-DMPIV_AB=1, Makefile) and left out of libmpiv.so, whose
// mpiv_debug_set refuses these values (the Python layer then switches to the A/B build).
bool ab_only(int o, int v) {
    switch (o) {
        case kOptRenderMv: case kOptRenderPair: case kOptSweepTile: return v != 0;
        case kOptRenderRing: return v > 0;
        case kOptRenderTile: return v != 0 && v != -1;
        case kOptRenderVshare: return v == -1 || v == 1;
        case kOptSweepStore: return v >= 0;
        case kOptRenderChunk: return v >= 100;
        case kOptSweepDlane: return v == 0;
        case kOptChunkRows: return v == 2 || v == 4;
        case kOptChunkFlight: return v == 4;
        case kOptChunkStrip: return v >= 2;
        case kOptSweepRows: return v == 6 || v == 8;
        case kOptBwdGather: return v == 1 || v == 2 || v == 3;
        case kOptBwdPollLimit: case kOptBwdFbBlocks: case kOptBwdFbMode: return v != 0;
        case kOptBwdOverlap: case kOptSweepBand: return v != 0;
        case kOptSweepPf: case kOptSweepSoa: return v > 0;
        default: return false;
    }
}

// mpiv_render_packed_census: set for the duration of one call on this thread; the rows-kernel
// launch takes it (and clears it) to launch the counting build
thread_local unsigned long long* g_census = nullptr;

// mpiv_route: set for the duration of one dry-run call on this thread; the entry point fills
// in the kernel (and grid size in work-items) it WOULD launch, and launches nothing
struct RouteNote {
    char name[160];
    int64_t threads;
};
thread_local RouteNote* g_route = nullptr;

int note_route(int64_t blocks_, int threads, const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_route->name, sizeof(g_route->name), fmt, ap);
    va_end(ap);
    g_route->threads = blocks_ * threads;
    return MPIV_OK;
}

constexpr int64_t kMaxGridYZ = 65535;
constexpr int kNativeLdsMaxP = 16;
constexpr int kChunkMaxLds = 65536;  // render_chunk_kernel: slots + P homographies, default LDS limit
constexpr int kChunkSplit = 1;       // composite phases per chunk (render_chunk.hip SPLIT)

constexpr int64_t kMaxGridX = 2147483647;

}  // namespace

using namespace mpiv;

namespace {

// rows per wave of render_chunk_kernel (chunk_rows option; automatic: 1)
int chunk_rows() {
    const int o = opt(kOptChunkRows);
    return (o == 2 || o == 4) ? o : 1;
}

// launch render_chunk_kernel<CH, SPLIT, R> with the block count of its 64 x 4R tiles
template <int CH, int SPLIT>
int launch_chunk(int R, const float* mpi, int64_t vstride, const RenderGeom& g, const ChunkGeom& cg, int B,
                 const float* homs, float* out, float4* ck, size_t lds, hipStream_t q, const char* nm) {
    const int64_t nb = (int64_t)blocks(g.W, kTileX) * blocks(g.H, kTileY * R) * B;
    if (nb > kMaxGridX) return fail(MPIV_ERR_ARG, "%s: too many blocks", nm);
    const int NT = (opt(kOptChunkFlight) == 4 && R == 1 && SPLIT == 1) ? 4 : 2;
    const int so = opt(kOptChunkStrip);
    if (CH == 8 && SPLIT == 1 && R == 1 && NT == 2 && so > 0) {  // 8 x SR strips, vertical tap reuse
        // 1: 8 x 16 strips, 2 rows in flight (production); A/B: 2 = 8 x 8, 3 = 8 x 8 with 3 rows in
        // flight, 4 = 8 x 16 with 3 (profiles/r04j_strips_ab.jsonl)
        const int SR = (so == 2 || so == 3) ? 8 : 16, SNT = so >= 3 ? 3 : 2;
        const int64_t ns = (int64_t)blocks(g.W, kStripTX) * blocks(g.H, SR) * B;
        if (ns > kMaxGridX) return fail(MPIV_ERR_ARG, "%s: too many blocks", nm);
        if (g_route) return note_route(ns, 256, "render_chunk_strip_kernel<%d, %d>", SR, SNT);
#if MPIV_AB
        if (so == 2)
            render_chunk_strip_kernel<8, 2><<<(unsigned)ns, 256, lds, q>>>(mpi, vstride, g, cg, B, homs, out, ck);
        else if (so == 3)
            render_chunk_strip_kernel<8, 3><<<(unsigned)ns, 256, lds, q>>>(mpi, vstride, g, cg, B, homs, out, ck);
        else if (so == 4)
            render_chunk_strip_kernel<16, 3><<<(unsigned)ns, 256, lds, q>>>(mpi, vstride, g, cg, B, homs, out, ck);
        else if (so == 5)  // homographies read through the caches instead of LDS: a fourth block per CU
            render_chunk_strip_kernel<16, 2><<<(unsigned)ns, 256, (size_t)chunk_slot_floats<8, 1>() * 4, q>>>(
                mpi, vstride, g, cg, B, homs, out, ck, 0);
        else
#endif
            render_chunk_strip_kernel<16, 2><<<(unsigned)ns, 256, lds, q>>>(mpi, vstride, g, cg, B, homs, out, ck);
        return launched(nm);
    }
    if (g_route) return note_route(nb, 256, "render_chunk_kernel<%d, %d, %d, %d>", CH, SPLIT, R, NT);
#if MPIV_AB  // R rows per wave / 4 sub-steps in flight: measured slower
    if (NT == 4)
        render_chunk_kernel<CH, SPLIT, 1, 4><<<(unsigned)nb, 256, lds, q>>>(mpi, vstride, g, cg, B, homs, out, ck);
    else if (R == 4)
        render_chunk_kernel<CH, SPLIT, SPLIT == 1 ? 4 : 1><<<(unsigned)nb, 256, lds, q>>>(mpi, vstride, g, cg, B, homs, out, ck);
    else if (R == 2)
        render_chunk_kernel<CH, SPLIT, SPLIT == 1 ? 2 : 1><<<(unsigned)nb, 256, lds, q>>>(mpi, vstride, g, cg, B, homs, out, ck);
    else
#endif
        render_chunk_kernel<CH, SPLIT, 1><<<(unsigned)nb, 256, lds, q>>>(mpi, vstride, g, cg, B, homs, out, ck);
    return launched(nm);
}

}  // namespace

extern "C" {

int mpiv_abi_version(void) { return MPIV_ABI_VERSION; }
const char* mpiv_last_error(void) { return g_err; }

#ifndef MPIV_SRC_HASH
#define MPIV_SRC_HASH "unknown"
#endif
const char* mpiv_build_id(void) { return MPIV_SRC_HASH; }

int mpiv_debug_set(const char* name, int value) {
    if (!name) return fail(MPIV_ERR_ARG, "mpiv_debug_set: null name");
    for (int i = 0; i < kNumOpts; ++i) {
        if (strcmp(name, kOptNames[i]) == 0) {
            if (!MPIV_AB && ab_only(i, value))
                return fail(MPIV_ERR_ARG, "mpiv_debug_set: %s=%d selects an A/B kernel, built only into libmpiv_ab.so",
                            name, value);
            __atomic_store_n(&g_opts[i], value, __ATOMIC_RELAXED);
            return MPIV_OK;
        }
    }
    if (strcmp(name, "reset") == 0) {
        for (int i = 0; i < kNumOpts; ++i) __atomic_store_n(&g_opts[i], kOptDefaults[i], __ATOMIC_RELAXED);
        return MPIV_OK;
    }
    return fail(MPIV_ERR_ARG, "mpiv_debug_set: unknown option '%s'", name);
}

int mpiv_render(const float* mpi, const int64_t st[5], int B, int H, int W, int P, const float* homs,
                float* out, void* stream) {
    if (!mpi || !st || !homs || !out) return fail(MPIV_ERR_ARG, "mpiv_render: null pointer");
    if (B <= 0 || H <= 0 || W <= 0 || P <= 0) return fail(MPIV_ERR_ARG, "mpiv_render: bad shape");
    if (B > kMaxGridYZ || (H + kTileY - 1) / kTileY > kMaxGridYZ) return fail(MPIV_ERR_ARG, "mpiv_render: too large");
    const NativeStrides s{st[0], st[1], st[2], st[3], st[4]};
    const dim3 grid(blocks(W, kTileX), blocks(H, kTileY), B);
    const RenderGeom g = make_geom(H, W, P);
    // 16-B vector texel loads when channels are contiguous and every texel is aligned
    const bool vec = s.c == 1 && aligned16(mpi) && s.b % 4 == 0 && s.y % 4 == 0 && s.x % 4 == 0 && s.p % 4 == 0;
    const bool fast = H >= 2 && W >= 2;
    hipStream_t q = S(stream);
    // in place at full-line coalescing (render_chunk.hip): planes contiguous per pixel
    // (s.p == 4), every offset from a chunk base below the buffer's out-of-range offset
    const int ch_opt = opt(kOptRenderChunk);
    const int CH = ch_opt > 0 ? ch_opt % 100 : (P <= 4 ? 4 : 8);
    const int SPLIT = ch_opt > 0 ? (ch_opt >= 100 ? 2 : 1) : kChunkSplit;
    const int64_t rec = ((int64_t)(H - 1) * s.y + (int64_t)(W - 1) * s.x) * 4 + CH * 16;
    const size_t ch_lds = (size_t)4 * (kWave / SPLIT) * (CH + 1) * 16 + (size_t)P * 36;
    if (vec && fast && s.p == 4 && ch_opt >= 0 && (CH == 4 || CH == 8) && rec < (int64_t)kOOB &&
        s.y / 4 < (1 << 22) && s.x / 4 < (1 << 22) && ch_lds <= (size_t)kChunkMaxLds) {
        const ChunkGeom cg{(int)(s.y / 4), (int)(s.x / 4), (int)rec};
        const int R = SPLIT == 1 ? chunk_rows() : 1;
#if MPIV_AB  // two composite phases per chunk (A/B)
        if (CH == 8 && SPLIT == 2)
            return launch_chunk<8, 2>(1, mpi, s.b, g, cg, B, homs, out, nullptr, ch_lds, q, "mpiv_render");
        if (SPLIT == 2)
            return launch_chunk<4, 2>(1, mpi, s.b, g, cg, B, homs, out, nullptr, ch_lds, q, "mpiv_render");
#endif
        if (CH == 8) return launch_chunk<8, 1>(R, mpi, s.b, g, cg, B, homs, out, nullptr, ch_lds, q, "mpiv_render");
        return launch_chunk<4, 1>(R, mpi, s.b, g, cg, B, homs, out, nullptr, ch_lds, q, "mpiv_render");
    }
    // footprints staged through LDS, read in place (render_lds.hip render_lds_native_kernel):
    // measured faster for few planes (P = 10: 0.031 vs 0.039 ms), slower for many (P = 128:
    // 2.78 vs 1.86 ms, the fills' 64-B segments no longer serve the next planes)
    if (vec && fast && P <= kNativeLdsMaxP && opt(kOptNativeLds)) {
        const int64_t nb = (int64_t)blocks(W, kLTX) * blocks(H, kLTY) * B;
        if (nb > kMaxGridX) return fail(MPIV_ERR_ARG, "mpiv_render: too many blocks");
        if (g_route) return note_route(nb, kLThreads, "render_lds_native_kernel<true>");
        render_lds_native_kernel<true><<<(unsigned)nb, kLThreads, 0, q>>>(mpi, s, g, B, homs, out);
        return launched("mpiv_render");
    }
    if (g_route)
        return note_route((int64_t)grid.x * grid.y * grid.z, 256, "render_native_kernel<%s, %s>", vec ? "true" : "false",
                          fast ? "true" : "false");
    if (vec && fast) render_native_kernel<true, true><<<grid, 256, 0, q>>>(mpi, s, g, homs, out);
    else if (vec) render_native_kernel<true, false><<<grid, 256, 0, q>>>(mpi, s, g, homs, out);
    else if (fast) render_native_kernel<false, true><<<grid, 256, 0, q>>>(mpi, s, g, homs, out);
    else render_native_kernel<false, false><<<grid, 256, 0, q>>>(mpi, s, g, homs, out);
    return launched("mpiv_render");
}

int mpiv_render_train(const float* mpi, const int64_t st[5], int B, int H, int W, int P, const float* homs,
                      float* out, float* ckpt, void* stream) {
    const char* nm = "mpiv_render_train";
    if (!mpi || !st || !homs || !out || !ckpt) return fail(MPIV_ERR_ARG, "%s: null pointer", nm);
    if (B <= 0 || H < 2 || W < 2 || P <= 0) return fail(MPIV_ERR_ARG, "%s: bad shape (H, W >= 2)", nm);
    const int64_t rec = ((int64_t)(H - 1) * st[1] + (int64_t)(W - 1) * st[2]) * 4 + 8 * 16;
    const size_t ch_lds = (size_t)4 * kWave * 9 * 16 + (size_t)P * 36;
    if (st[4] != 1 || st[3] != 4 || st[0] % 4 || st[1] % 4 || st[2] % 4 || st[1] < 0 || st[2] < 0 ||
        !aligned16(mpi) || !aligned16(ckpt) || rec >= (int64_t)kOOB || st[1] / 4 >= (1 << 22) ||
        st[2] / 4 >= (1 << 22) || ch_lds > (size_t)kChunkMaxLds)
        return fail(MPIV_ERR_ARG, "%s: rgba_layers must be read in place (16-byte texels, planes contiguous per "
                    "pixel, one view below 2 GiB, P <= 796)", nm);
    const ChunkGeom cg{(int)(st[1] / 4), (int)(st[2] / 4), (int)rec};
    return launch_chunk<8, 1>(chunk_rows(), mpi, st[0], make_geom(H, W, P), cg, B, homs, out,
                              reinterpret_cast<float4*>(ckpt), ch_lds, S(stream), nm);
}

int mpiv_pack_planes(const float* mpi, const int64_t st[4], int H, int W, int P, float* packed, void* stream) {
    if (!mpi || !st || !packed) return fail(MPIV_ERR_ARG, "mpiv_pack_planes: null pointer");
    if (H <= 0 || W <= 0 || P <= 0) return fail(MPIV_ERR_ARG, "mpiv_pack_planes: bad shape");
    if (!aligned16(packed)) return fail(MPIV_ERR_ARG, "mpiv_pack_planes: packed must be 16-byte aligned");
    if ((int64_t)(H + 2 * kPad) * (W + 2 * kPad) * 16 >= (int64_t)kOOB)
        return fail(MPIV_ERR_ARG, "mpiv_pack_planes: padded plane larger than 2 GiB");
    const int64_t npix = (int64_t)(H + 2 * kPad) * (W + 2 * kPad);
    if (blocks(P, kPackPl) > kMaxGridYZ) return fail(MPIV_ERR_ARG, "mpiv_pack_planes: too many planes");
    const NativeStrides s{0, st[0], st[1], st[2], st[3]};
    dim3 grid(blocks(npix, kPackPix), blocks(P, kPackPl), 1);
    pack_planes_kernel<<<grid, 256, 0, S(stream)>>>(mpi, s, H, W, P, make_fastdiv((unsigned)(W + 2 * kPad)),
                                                    reinterpret_cast<float4*>(packed), npix);
    return launched("mpiv_pack_planes");
}

// variant 0: direct gathers (render_packed_kernel, the default); 1: LDS-staged footprints
// Same-row tap reuse (render.hip SAME): automatic where the sample advances at most 0.8 texel rows
// per output row (the reference's swapped y / (W-1) normalisation on landscape frames: configs 2, 5);
// render_same=-1 turns it off, 1 forces it on.
static bool rows_same(float syr) {
    const int o = opt(kOptRenderSame);
    return o > 0 || (o == 0 && syr <= 0.8f);
}

// ... and its out-of-range south loads on rows where every lane stayed (render.hip OOB): automatic
// for launches of one or two views; render_same=2 forces them, 1 keeps the plain same-row kernel.
static bool rows_same_oob(int V) {
    const int o = opt(kOptRenderSame);
    return o == 2 || (o == 0 && V <= 2);
}

static int render_packed_impl(const float* packed, int H, int W, int P, int p_begin, int p_end, int back,
                              const float* homs, int V, float* out, bool ct, int variant, void* stream) {
    const char* nm = ct ? "mpiv_render_packed_ct" : "mpiv_render_packed";
    if (!packed || !homs || !out) return fail(MPIV_ERR_ARG, "%s: null pointer", nm);
    if (V <= 0 || H <= 0 || W <= 0 || P <= 0) return fail(MPIV_ERR_ARG, "%s: bad shape", nm);
    if (p_begin < 0 || p_end > P || p_begin >= p_end) return fail(MPIV_ERR_ARG, "%s: bad plane range", nm);
    if (!aligned16(packed) || (ct && !aligned16(out))) return fail(MPIV_ERR_ARG, "%s: 16-byte alignment", nm);
    if ((int64_t)(H + 2 * kPad) * (W + 2 * kPad) * 16 >= (int64_t)kOOB || H >= (1 << 22) || W >= (1 << 22))
        return fail(MPIV_ERR_ARG, "%s: padded plane larger than 2 GiB or a side >= 2^22", nm);
    const float4* pk = reinterpret_cast<const float4*>(packed);
    const int64_t ps = (int64_t)(H + 2 * kPad) * (W + 2 * kPad);
    const RenderGeom g = make_geom(H, W, P);
    const bool fast = H >= 2 && W >= 2;  // div_const needs divisors >= 1
    hipStream_t st = S(stream);
#if MPIV_AB
    if (variant == 1 && fast && p_end - p_begin <= kLMaxP) {
        // footprints staged through LDS (render_lds.hip)
        const int64_t nb = (int64_t)blocks(W, kLTX) * blocks(H, kLTY) * V;
        if (nb > kMaxGridX) return fail(MPIV_ERR_ARG, "%s: too many blocks", nm);
        const dim3 grid((unsigned)nb), blk(kLThreads);
        if (ct)
            render_lds_kernel<true, true><<<grid, blk, 0, st>>>(pk, ps, g, V, p_begin, p_end, back, homs, out);
        else
            render_lds_kernel<false, true><<<grid, blk, 0, st>>>(pk, ps, g, V, p_begin, p_end, 1, homs, out);
        return launched(nm);
    }
    // several views of one MPI: the multi-view LDS-staged kernel (render_mv.hip) on request
    // (A/B: it ties the direct kernel on a camera path)
    if (variant == 0 && fast && V >= kMMinViews && p_end - p_begin <= kMMaxP && opt(kOptRenderMv)) {
        const int64_t nb = (int64_t)blocks(W, kMTX) * blocks(H, kMTY) * ((V + kMVB - 1) / kMVB);
        if (nb > kMaxGridX) return fail(MPIV_ERR_ARG, "%s: too many blocks", nm);
        const int shrink = opt(kOptBoxShrink);
        const dim3 grid((unsigned)nb), blk(kMThreads);
        if (ct)
            render_mv_kernel<true><<<grid, blk, 0, st>>>(pk, ps, g, V, p_begin, p_end, back, shrink, homs, out);
        else
            render_mv_kernel<false><<<grid, blk, 0, st>>>(pk, ps, g, V, p_begin, p_end, 1, shrink, homs, out);
        return launched(nm);
    }
    // LDS-DMA ring (render_ring.hip): footprints streamed into LDS several planes ahead
    // opt-in A/B only: measured back to back, the ring ties the direct kernel on single views
    // (0.47 ms both) and loses on multi-view launches and stretched footprints
    if (const int ring = (variant == 0 && fast && p_end - p_begin <= kRMaxP) ? opt(kOptRenderRing) : -1;
        ring > 0) {
        // ring geometry: {waves, rows per lane, slots, fills per wave and plane}
        static const int kRingGeo[][4] = {{4, 2, 4, 4}, {4, 4, 3, 5}, {4, 2, 3, 4}, {8, 1, 2, 2},
                                          {8, 1, 3, 2}, {8, 1, 4, 2}, {8, 2, 2, 3}, {16, 1, 2, 2}};
        if (ring > 8) return fail(MPIV_ERR_ARG, "%s: unknown ring geometry %d", nm, ring);
        const int* geo = kRingGeo[ring - 1];
        const int ty = geo[0] * geo[1];
        const int64_t nb = (int64_t)blocks(W, kRTX) * blocks(H, ty) * V;
        if (nb > kMaxGridX) return fail(MPIV_ERR_ARG, "%s: too many blocks", nm);
#define MPIV_RING(NW, RPL, NS, F)                                                                                \
    if (ct)                                                                                                     \
        render_ring_kernel<true, NW, RPL, NS, F><<<(unsigned)nb, NW * 64, 0, st>>>(pk, ps, g, V, p_begin, p_end, \
                                                                                   back, homs, out);           \
    else                                                                                                        \
        render_ring_kernel<false, NW, RPL, NS, F><<<(unsigned)nb, NW * 64, 0, st>>>(pk, ps, g, V, p_begin, p_end, 1, \
                                                                                    homs, out)
        switch (ring) {
            case 1: MPIV_RING(4, 2, 4, 4); break;
            case 2: MPIV_RING(4, 4, 3, 5); break;
            case 3: MPIV_RING(4, 2, 3, 4); break;
            case 4: MPIV_RING(8, 1, 2, 2); break;
            case 5: MPIV_RING(8, 1, 3, 2); break;
            case 6: MPIV_RING(8, 1, 4, 2); break;
            case 7: MPIV_RING(8, 2, 2, 3); break;
            default: MPIV_RING(16, 1, 2, 2); break;
        }
#undef MPIV_RING
        return launched(nm);
    }
    // pixel pairs sharing their common taps (render.hip render_pair_kernel): opt-in A/B,
    // 20 % fewer gathers but 117 VGPRs (4 waves/SIMD), measured 3 % slower
    if (const int pair = fast ? opt(kOptRenderPair) : 0) {  // 1: two planes in flight, 2: one
        const int64_t nb = (int64_t)blocks(W, kPairX) * blocks(H, kTileY) * V;
        if (nb > kMaxGridX) return fail(MPIV_ERR_ARG, "%s: too many blocks", nm);
        if (ct && pair == 1)
            render_pair_kernel<true, true><<<(unsigned)nb, 256, 0, st>>>(pk, ps, g, V, p_begin, p_end, back, homs, out);
        else if (ct)
            render_pair_kernel<true, false><<<(unsigned)nb, 256, 0, st>>>(pk, ps, g, V, p_begin, p_end, back, homs, out);
        else if (pair == 1)
            render_pair_kernel<false, true><<<(unsigned)nb, 256, 0, st>>>(pk, ps, g, V, p_begin, p_end, 1, homs, out);
        else
            render_pair_kernel<false, false><<<(unsigned)nb, 256, 0, st>>>(pk, ps, g, V, p_begin, p_end, 1, homs, out);
        return launched(nm);
    }
#endif  // MPIV_AB

    // R rows per work-item, planes outermost (render.hip render_rows_kernel), automatic
    // (bench_configs.py A/B, profiles/r02_vshare_ab.txt), all with vertical tap reuse and a ring
    // of D rows in flight:
    //  * one or two views (HBM-bound): R = 4, D = 4 (single view 0.383 ms vs 0.40-0.41 for (8, 4),
    //    0.44 for plain R = 8, 0.48-0.51 for the one-row kernel; config-5 shard 0.776 vs 0.80);
    //  * 3 to 8 views: R = 8, D = 4 (8 views 1.80-1.87 vs 1.93-1.98 ms with D = 2, 1.90 for (4, 4));
    //  * more views (the texture path binds): near-square MPIs R = 6, D = 3 (125 views 26.5-26.9
    //    vs 27.4-28.3 ms with D = 2, 30.8 without reuse); stretched MPIs R = 9, D = 3 (config 2 at
    //    64 views 2.04-2.09 vs 2.11-2.17 ms for (8, 4), 2.33-2.39 one-row);
    //  * stretched MPIs (the reference's swapped x/(H-1), y/(W-1) normalisation: footprints
    //    stretched by W/(H-1) and H/(W-1)) only when the tiles fill the chip (>= 2048 blocks of
    //    64x32): config 5's plane shard 0.80 vs 0.87 ms one-row; config 2 at one view (288
    //    blocks) is latency-bound (0.079 vs 0.054 ms), so the one-row kernel keeps small launches;
    //  * round 6: where the sample advances <= 0.8 texel rows per output row (configs 2 and 5),
    //    same-row tap reuse with R = 6, D = 3 at every view count (profiles/r06_same_ab*.jsonl:
    //    config-5 shard 0.655-0.67 vs 0.77-0.78 ms, config 2 at 64 views 1.95-1.96 vs 2.05, at
    //    8 views 0.253-0.256 vs 0.26-0.27).
    const float sxr = (float)W / (float)(H > 1 ? H - 1 : 1), syr = (float)H / (float)(W > 1 ? W - 1 : 1);
    const bool square = sxr >= 0.8f && sxr <= 1.25f && syr >= 0.8f && syr <= 1.25f;
    const int rows_opt = opt(kOptRenderTile);
    const int64_t rows_blocks = (int64_t)blocks(W, kTileX) * blocks(H, 4 * 8) * V;
    const bool stretched_vs = !square && rows_blocks >= 2048;
    const bool variants_off = !opt(kOptRenderMv) && !opt(kOptRenderPair);
    const int rows_auto = ((square || stretched_vs) && variants_off) ? 8 : 0;
    const int vs_opt = opt(kOptRenderVshare);
    [[maybe_unused]] const int rows_sel = fast ? (rows_opt ? rows_opt : rows_auto) : 0;
#if MPIV_AB
    if (const int rows = rows_sel; rows == 108 || rows == 116 || rows == 132) {
        // R rows with the compositing state in LDS (render_rows_lds_kernel)
        const int R = rows - 100;
        const int64_t nb = (int64_t)blocks(W, kTileX) * blocks(H, 4 * R) * V;
        if (nb > kMaxGridX) return fail(MPIV_ERR_ARG, "%s: too many blocks", nm);
#define MPIV_ROWSL(R)                                                                                                  \
    if (ct)                                                                                                           \
        render_rows_lds_kernel<true, R><<<(unsigned)nb, 256, 0, st>>>(pk, ps, g, V, p_begin, p_end, back, homs, out); \
    else                                                                                                              \
        render_rows_lds_kernel<false, R><<<(unsigned)nb, 256, 0, st>>>(pk, ps, g, V, p_begin, p_end, 1, homs, out)
        if (R == 8) MPIV_ROWSL(8);
        else if (R == 16) MPIV_ROWSL(16);
        else MPIV_ROWSL(32);
#undef MPIV_ROWSL
        return launched(nm);
    }
#endif  // MPIV_AB

    // vertical tap reuse with D rows in flight; render_vshare forces one of the automatic
    // choices: 3: (R, D) = (8, 4), 4: (6, 3), 5: (9, 3), 11: (4, 4) (the other (R, D) points of
    // profiles/r02_vshare_ab.txt were A/B builds and are not shipped)
    int vsd = 0;
    if (fast && (vs_opt == 3 || vs_opt == 4 || vs_opt == 5 || vs_opt == 11))
        vsd = vs_opt;
    else if (fast && vs_opt == 0 && !rows_opt && rows_auto == 8)
        vsd = rows_same(syr) ? 4 : V <= 2 ? 11 : V <= 8 ? 3 : square ? 4 : 5;
    if (vsd) {
        const int R = vsd == 3 ? 8 : vsd == 4 ? 6 : vsd == 5 ? 9 : 4;
        const int64_t nb = (int64_t)blocks(W, kTileX) * blocks(H, 4 * R) * V;
        if (nb > kMaxGridX) return fail(MPIV_ERR_ARG, "%s: too many blocks", nm);
        // same-row tap reuse (round 6) where the sample advances less than a texel row per output row
        const bool same = rows_same(syr);
        const bool oob = same && vsd == 4 && rows_same_oob(V);  // R = 6 only
        // the counting build (mpiv_render_packed_census) exists for the automatic choices
        if (g_route)
            return note_route(nb, 256, "render_rows_kernel<%s, %d, true, false, %d, %s, %s>", ct ? "true" : "false", R,
                              vsd == 3 || vsd == 11 ? 4 : 3, same ? "true" : "false", oob ? "true" : "false");
        unsigned long long* cn = (g_census && !ct) ? g_census : nullptr;
        if (cn) g_census = nullptr;
#define MPIV_VSD(R, D, SM, OB)                                                                                        \
    if (ct)                                                                                                          \
        render_rows_kernel<true, R, true, false, D, SM, OB><<<(unsigned)nb, 256, 0, st>>>(pk, ps, g, V, p_begin,     \
                                                                                           p_end, back, homs, out);  \
    else                                                                                                             \
        render_rows_kernel<false, R, true, false, D, SM, OB><<<(unsigned)nb, 256, 0, st>>>(pk, ps, g, V, p_begin,    \
                                                                                            p_end, 1, homs, out)
#define MPIV_VSDC(R, D, SM, OB)                                                                                       \
    if (cn)                                                                                                          \
        render_rows_kernel<false, R, true, true, D, SM, OB><<<(unsigned)nb, 256, 0, st>>>(pk, ps, g, V, p_begin,     \
                                                                                          p_end, 1, homs, out, cn);  \
    else                                                                                                             \
        MPIV_VSD(R, D, SM, OB)
        if (oob) {
            MPIV_VSDC(6, 3, true, true);
        } else if (same) {
            switch (vsd) {
                case 3: MPIV_VSDC(8, 4, true, false); break;
                case 4: MPIV_VSDC(6, 3, true, false); break;
                case 5: MPIV_VSDC(9, 3, true, false); break;
                default: MPIV_VSDC(4, 4, true, false); break;
            }
        } else {
            switch (vsd) {
                case 3: MPIV_VSDC(8, 4, false, false); break;
                case 4: MPIV_VSDC(6, 3, false, false); break;
                case 5: MPIV_VSDC(9, 3, false, false); break;
                default: MPIV_VSDC(4, 4, false, false); break;
            }
        }
#undef MPIV_VSDC
#undef MPIV_VSD
        return launched(nm);
    }
#if MPIV_AB
    if (const int rows = rows_sel; rows == 2 || rows == 4 || rows == 8 || rows == 16) {
        const int64_t nb = (int64_t)blocks(W, kTileX) * blocks(H, 4 * rows) * V;
        if (nb > kMaxGridX) return fail(MPIV_ERR_ARG, "%s: too many blocks", nm);
#define MPIV_ROWS(R)                                                                                               \
    if (ct)                                                                                                       \
        render_rows_kernel<true, R><<<(unsigned)nb, 256, 0, st>>>(pk, ps, g, V, p_begin, p_end, back, homs, out); \
    else                                                                                                          \
        render_rows_kernel<false, R><<<(unsigned)nb, 256, 0, st>>>(pk, ps, g, V, p_begin, p_end, 1, homs, out)
        const bool vs = vs_opt == 1;  // two rows in flight (A/B; the automatic routes are above)
        if (rows == 2) MPIV_ROWS(2);
        else if (rows == 4) MPIV_ROWS(4);
        else if (rows == 8 && g_census && !ct) {  // the counting build (mpiv_render_packed_census)
            unsigned long long* cn = g_census;
            g_census = nullptr;
            if (vs)
                render_rows_kernel<false, 8, true, true><<<(unsigned)nb, 256, 0, st>>>(pk, ps, g, V, p_begin, p_end, 1,
                                                                                       homs, out, cn);
            else
                render_rows_kernel<false, 8, false, true><<<(unsigned)nb, 256, 0, st>>>(pk, ps, g, V, p_begin, p_end,
                                                                                        1, homs, out, cn);
        } else if (rows == 8 && vs) {
            if (ct)
                render_rows_kernel<true, 8, true><<<(unsigned)nb, 256, 0, st>>>(pk, ps, g, V, p_begin, p_end, back, homs,
                                                                                 out);
            else
                render_rows_kernel<false, 8, true><<<(unsigned)nb, 256, 0, st>>>(pk, ps, g, V, p_begin, p_end, 1, homs,
                                                                                  out);
        } else if (rows == 8) MPIV_ROWS(8);
        else MPIV_ROWS(16);
#undef MPIV_ROWS
        return launched(nm);
    }
#endif  // MPIV_AB

    const int64_t nblocks = (int64_t)blocks(W, kTileX) * blocks(H, kTileY) * V;
    if (nblocks > kMaxGridX) return fail(MPIV_ERR_ARG, "%s: too many blocks", nm);
    const dim3 grid((unsigned)nblocks), blk(256);
    if (g_route)
        return note_route(nblocks, 256, "render_packed_kernel<%s, %s>", ct ? "true" : "false", fast ? "true" : "false");
    if (ct && fast)
        render_packed_kernel<true, true><<<grid, blk, 0, st>>>(pk, ps, g, V, p_begin, p_end, back, homs, out);
    else if (ct)
        render_packed_kernel<true, false><<<grid, blk, 0, st>>>(pk, ps, g, V, p_begin, p_end, back, homs, out);
    else if (fast)
        render_packed_kernel<false, true><<<grid, blk, 0, st>>>(pk, ps, g, V, p_begin, p_end, 1, homs, out);
    else
        render_packed_kernel<false, false><<<grid, blk, 0, st>>>(pk, ps, g, V, p_begin, p_end, 1, homs, out);
    return launched(nm);
}

int mpiv_render_packed(const float* packed, int H, int W, int P, const float* homs, int V, float* out,
                       void* stream) {
    return render_packed_impl(packed, H, W, P, 0, P, 1, homs, V, out, false, 0, stream);
}

int mpiv_render_packed_census(const float* packed, int H, int W, int P, const float* homs, int V, float* out,
                              unsigned long long* census, void* stream) {
    if (!census) return fail(MPIV_ERR_ARG, "mpiv_render_packed_census: null census");
    g_census = census;  // render_packed_impl launches the counting build of the rows kernel
    const int rc = render_packed_impl(packed, H, W, P, 0, P, 1, homs, V, out, false, 0, stream);
    const bool used = g_census == nullptr;
    g_census = nullptr;
    if (rc != MPIV_OK) return rc;
    if (!used) return fail(MPIV_ERR_ARG, "mpiv_render_packed_census: this launch does not route to render_rows_kernel");
    return MPIV_OK;
}

int mpiv_render_packed_lds(const float* packed, int H, int W, int P, const float* homs, int V, float* out,
                           void* stream) {
#if !MPIV_AB
    (void)packed, (void)H, (void)W, (void)P, (void)homs, (void)V, (void)out, (void)stream;
    return fail(MPIV_ERR_ARG, "mpiv_render_packed_lds: an A/B kernel, built only into libmpiv_ab.so");
#endif
    return render_packed_impl(packed, H, W, P, 0, P, 1, homs, V, out, false, 1, stream);
}

int mpiv_render_packed_ct(const float* packed, int H, int W, int P, int p_begin, int p_end, int back,
                          const float* homs, int V, float* ct, void* stream) {
    return render_packed_impl(packed, H, W, P, p_begin, p_end, back, homs, V, ct, true, 0, stream);
}

// Rows [y_begin, y_end) of mpiv_render_packed_ct's partial: the plane-sharded render issues its
// G row bands one launch each, so band k can leave for rank k while the next band renders
// (parallel.py).  Always the rows kernel with vertical tap reuse (every render route gives the
// same bits), its (R, rows in flight) chosen as the full-frame route chooses them.
int mpiv_render_packed_ct_rows(const float* packed, int H, int W, int P, int p_begin, int p_end, int back,
                               const float* homs, int V, int y_begin, int y_end, float* ct, void* stream) {
    const char* nm = "mpiv_render_packed_ct_rows";
    if (!packed || !homs || !ct) return fail(MPIV_ERR_ARG, "%s: null pointer", nm);
    if (V <= 0 || H < 2 || W < 2 || P <= 0) return fail(MPIV_ERR_ARG, "%s: bad shape (H, W >= 2)", nm);
    if (p_begin < 0 || p_end > P || p_begin >= p_end) return fail(MPIV_ERR_ARG, "%s: bad plane range", nm);
    if (y_begin < 0 || y_end > H || y_begin >= y_end) return fail(MPIV_ERR_ARG, "%s: bad row range", nm);
    if (!aligned16(packed) || !aligned16(ct)) return fail(MPIV_ERR_ARG, "%s: 16-byte alignment", nm);
    if ((int64_t)(H + 2 * kPad) * (W + 2 * kPad) * 16 >= (int64_t)kOOB || H >= (1 << 22) || W >= (1 << 22))
        return fail(MPIV_ERR_ARG, "%s: padded plane larger than 2 GiB or a side >= 2^22", nm);
    const float4* pk = reinterpret_cast<const float4*>(packed);
    const int64_t ps = (int64_t)(H + 2 * kPad) * (W + 2 * kPad);
    const RenderGeom g = make_geom(H, W, P);
    const float sxr = (float)W / (float)(H - 1), syr = (float)H / (float)(W - 1);
    const bool square = sxr >= 0.8f && sxr <= 1.25f && syr >= 0.8f && syr <= 1.25f;
    const bool same = rows_same(syr);
    const bool oob = same && rows_same_oob(V);
    const int R = same ? 6 : V <= 2 ? 4 : V <= 8 ? 8 : square ? 6 : 9;
    const int64_t nb = (int64_t)blocks(W, kTileX) * blocks(y_end - y_begin, 4 * R) * V;
    if (nb > kMaxGridX) return fail(MPIV_ERR_ARG, "%s: too many blocks", nm);
    if (g_route)
        return note_route(nb, 256, "render_rows_kernel<true, %d, true, false, %d, %s, %s>", R, R == 4 || R == 8 ? 4 : 3,
                          same ? "true" : "false", oob ? "true" : "false");
    hipStream_t st = S(stream);
#define MPIV_CTR(RR, DD, SM)                                                                                           \
    render_rows_kernel<true, RR, true, false, DD, SM><<<(unsigned)nb, 256, 0, st>>>(pk, ps, g, V, p_begin, p_end, back, \
                                                                                    homs, ct, nullptr, y_begin, y_end)
    if (oob) {
        render_rows_kernel<true, 6, true, false, 3, true, true><<<(unsigned)nb, 256, 0, st>>>(
            pk, ps, g, V, p_begin, p_end, back, homs, ct, nullptr, y_begin, y_end);
    } else if (same) {
        switch (R) {
            case 4: MPIV_CTR(4, 4, true); break;
            case 8: MPIV_CTR(8, 4, true); break;
            case 6: MPIV_CTR(6, 3, true); break;
            default: MPIV_CTR(9, 3, true); break;
        }
    } else {
        switch (R) {
            case 4: MPIV_CTR(4, 4, false); break;
            case 8: MPIV_CTR(8, 4, false); break;
            case 6: MPIV_CTR(6, 3, false); break;
            default: MPIV_CTR(9, 3, false); break;
        }
    }
#undef MPIV_CTR
    return launched(nm);
}

// ---- render backward (render_bwd.hip) ----------------------------------------------

namespace {

inline size_t align256(size_t n) { return (n + 255) & ~(size_t)255; }

// Planes per group (round 4): all of them up to 2^25 plane-pixels, else the fewest equal groups
// below that, rounded up to whole 8-plane chunks.  A view's backward runs group by group, back
// to front (chain -> gather -> check -> fallback per group, the running g handed down in
// gbuf), so the workspace holds the d samples of one group (config 4: 32 of 128 planes, 0.54 GB
// instead of 2.15) and the fallback's bucket arrays are sized for one group too.
int bwd_group_planes(int H, int W, int P) {
    const int64_t n = (int64_t)P * H * W, cap = (int64_t)1 << 25;
    if (H < 2 || W < 2) return P;  // degenerate frames take the generic recipe, one group
    if (opt(kOptBwdGroup) > 0) return std::min(P, (opt(kOptBwdGroup) + kBwdCH - 1) / kBwdCH * kBwdCH);
    if (n <= cap) return P;
    const int64_t groups = (n + cap - 1) / cap;
    const int gp = (int)(((int64_t)P + groups - 1) / groups);
    return std::min(P, (gp + kBwdCH - 1) / kBwdCH * kBwdCH);
}

// workspace carve-up for one view; returns the total size in bytes
// (the counters and flags first: _lib.bwd_flag_offset mirrors their offsets; gbuf: the running
// over-composite adjoint g handed from one plane group to the next, also the frame scratch of the
// forward that fills ckpt when the caller has no checkpoints and the view has several groups)
// dsp: planes whose d samples are resident (P: one group; bwd_group_planes: the smallest); the
// fallback's bucket arrays always take one group of bwd_group_planes (its plane chunk)
// nwin: d-sample windows (2: the overlapped schedule, mpiv_render_backward -- group k's gather reads
// one window while group k-1's chain fills the other; each window has its own counters, ws2)
size_t bwd_layout(int H, int W, int P, int dsp, char* base, BwdWs* ws, float4** gbuf = nullptr, int nwin = 1,
                  BwdWs* ws2 = nullptr) {
    const size_t hw = (size_t)H * W;
    const int pc = bwd_group_planes(H, W, P);
    const size_t nk = (size_t)pc * (H + 1) * (W + 1);
    const size_t nb = (nk + kScanTile - 1) / kScanTile;
    const size_t nchunk = (size_t)(P + kBwdCH - 1) / kBwdCH;
    size_t off = 0;
    auto take = [&](size_t bytes) {
        char* p = base ? base + off : nullptr;
        off += align256(bytes);
        return p;
    };
    char* truth = take(kCtrSlots * 8);
    char* found = take(kCtrSlots * 8);
    char* flag = take(64);  // 16 words: [0..4] check / fallback, [8], [9] block-exit counters
    char* truth2 = take(nwin > 1 ? kCtrSlots * 8 : 0);  // the second window's counters (same carve-up)
    char* found2 = take(nwin > 1 ? kCtrSlots * 8 : 0);
    char* flag2 = take(nwin > 1 ? 64 : 0);
    char* ds = take((size_t)nwin * dsp * hw * 16);
    char* ckpt = take(nchunk * hw * 16);
    char* inv = take((size_t)P * 12 * 4);
    char* gb = take(dsp < P ? hw * 16 : 0);
    if (gbuf) *gbuf = reinterpret_cast<float4*>(gb);
    const size_t ntiles = (size_t)((W + kGTW - 1) / kGTW) * ((H + kGTY - 1) / kGTY);
    char* box = take((size_t)P * ntiles * 16);
    char* key = take((size_t)pc * hw * 4);
    char* count = take(nk * 4);
    char* offs = take((nk + 1) * 4);
    char* ids = take((size_t)pc * hw * 4);
    char* bsum = take(nb * 4);
    char* big = take(((size_t)pc * hw / (kSmallBucket + 1) + 2) * 4);
    if (ws) {
        ws->ds = reinterpret_cast<float4*>(ds);
        ws->ckpt = reinterpret_cast<float4*>(ckpt);
        ws->inv = reinterpret_cast<float*>(inv);
        ws->truth = reinterpret_cast<unsigned long long*>(truth);
        ws->found = reinterpret_cast<unsigned long long*>(found);
        ws->flag = reinterpret_cast<int*>(flag);
        ws->box = reinterpret_cast<int4*>(box);
        ws->pc = pc;
        ws->key = reinterpret_cast<int*>(key);
        ws->count = reinterpret_cast<int*>(count);
        ws->offs = reinterpret_cast<int*>(offs);
        ws->ids = reinterpret_cast<int*>(ids);
        ws->bsum = reinterpret_cast<int*>(bsum);
        ws->big = reinterpret_cast<int*>(big);
        ws->vcount = ws->flag + 4;
        if (ws2) {
            *ws2 = *ws;
            ws2->ds = reinterpret_cast<float4*>(ds + (size_t)dsp * hw * 16);
            ws2->truth = reinterpret_cast<unsigned long long*>(truth2);
            ws2->found = reinterpret_cast<unsigned long long*>(found2);
            ws2->flag = reinterpret_cast<int*>(flag2);
        }
    }
    return off;
}

// The overlapped backward's second stream and its events, per device (created on first use; the
// schedule's enqueue runs under g_aux_mu, so concurrent callers never interleave their records
// and waits on the shared events)
struct BwdAux {
    hipStream_t s = nullptr;
    hipEvent_t chain[2] = {}, done[2] = {}, view = nullptr;
    bool ok = false, tried = false;
};
BwdAux g_aux[64];
std::mutex g_aux_mu;

BwdAux* bwd_aux(int dev) {  // call with g_aux_mu held
    BwdAux& a = g_aux[dev];
    if (!a.tried) {
        a.tried = true;
        a.ok = hipStreamCreateWithFlags(&a.s, hipStreamNonBlocking) == hipSuccess;
        for (int i = 0; i < 2 && a.ok; ++i)
            a.ok = hipEventCreateWithFlags(&a.chain[i], hipEventDisableTiming) == hipSuccess &&
                   hipEventCreateWithFlags(&a.done[i], hipEventDisableTiming) == hipSuccess;
        a.ok = a.ok && hipEventCreateWithFlags(&a.view, hipEventDisableTiming) == hipSuccess;
    }
    return a.ok ? &a : nullptr;
}


}  // namespace

// one plane group (every plane's d samples resident: the fastest schedule), unless the
// bwd_group test hook asks for groups
size_t mpiv_render_backward_workspace_size(int H, int W, int P) {
    if (H <= 0 || W <= 0 || P <= 0) return 0;
    // the one-group schedule's, or (bwd_group test hook) one window of that group size; with room for
    // the overlapped schedule's two windows when it is selected (A/B build, bwd_overlap=1)
    const size_t one = bwd_layout(H, W, P, opt(kOptBwdGroup) > 0 ? bwd_group_planes(H, W, P) : P, nullptr, nullptr);
    const int gp = bwd_group_planes(H, W, P);
    return MPIV_AB && opt(kOptBwdOverlap) != 0 && gp < P
               ? std::max(one, bwd_layout(H, W, P, gp, nullptr, nullptr, nullptr, 2)) : one;
}

// the smallest workspace: plane groups of bwd_group_planes (config 4: 1.3 GB instead of 3.0)
size_t mpiv_render_backward_workspace_size_min(int H, int W, int P) {
    if (H <= 0 || W <= 0 || P <= 0) return 0;
    return bwd_layout(H, W, P, bwd_group_planes(H, W, P), nullptr, nullptr);
}

// Page-locked, device-mapped abort flags, one word per device (allocated once per process, fine-grained:
// a device store is visible to the host without a copy).  The backward's NaN fill of an aborted view sets
// the device's word to 1; the Python layer reads and clears it on the host (_lib._AbortMonitor) -- no
// per-call copy, event or synchronisation.
static int* g_abort_host = nullptr;
static int* g_abort_dev = nullptr;
static std::once_flag g_abort_once;
constexpr int kAbortSlots = 64;

static int* abort_flags_dev() {
    std::call_once(g_abort_once, []() {
        void* h = nullptr;
        if (hipHostMalloc(&h, kAbortSlots * sizeof(int), hipHostMallocMapped | hipHostMallocPortable |
                                                              hipHostMallocCoherent) != hipSuccess || !h)
            return;
        std::memset(h, 0, kAbortSlots * sizeof(int));
        void* d = nullptr;
        if (hipHostGetDevicePointer(&d, h, 0) != hipSuccess || !d) return;
        g_abort_host = static_cast<int*>(h);
        g_abort_dev = static_cast<int*>(d);
    });
    return g_abort_dev;
}

int* mpiv_render_backward_abort_flag(int device) {
    if (device < 0 || device >= kAbortSlots) return nullptr;
    abort_flags_dev();
    return g_abort_host ? g_abort_host + device : nullptr;
}

constexpr int64_t kFoldCheckMaxBlocks = 8192;  // gather grids up to this size run the check in their last block

static int render_backward_impl(const char* nm, const float* mpi, const int64_t st[5], int V, int H, int W, int P,
                                const float* homs, const float* dout, const float* ckpt, float* dmpi, void* workspace,
                                size_t ws_bytes, void* stream, bool watched) {
    if (!mpi || !st || !homs || !dout || !dmpi || !workspace) return fail(MPIV_ERR_ARG, "%s: null pointer", nm);
    if (V <= 0 || H <= 0 || W <= 0 || P <= 0) return fail(MPIV_ERR_ARG, "%s: bad shape", nm);
    // in place: planes contiguous per pixel (16-B texels), every tap below the buffer range
    const int64_t rec = ((int64_t)(H - 1) * st[1] + (int64_t)(W - 1) * st[2]) * 4 + kBwdCH * 16;
    if (st[4] != 1 || st[3] != 4 || st[0] % 4 || st[1] % 4 || st[2] % 4 || !aligned16(mpi))
        return fail(MPIV_ERR_ARG, "%s: rgba_layers must have 16-byte aligned texels with planes contiguous per pixel "
                    "(strides[3] == 4, strides[4] == 1)", nm);
    if (st[1] < 0 || st[2] < 0 || rec >= (int64_t)kOOB || st[1] / 4 >= (1 << 22) || st[2] / 4 >= (1 << 22))
        return fail(MPIV_ERR_ARG, "%s: one view's MPI must span less than 2 GiB", nm);
    // the chain's homographies go to LDS beside its sample slots when they fit (P <= 796),
    // else it reads them from global memory
    const size_t slots_lds = (size_t)4 * kWave * (kBwdCH + 1) * 16;
    const int h_lds = slots_lds + (size_t)P * 36 <= (size_t)kChunkMaxLds;
    const size_t chain_lds = slots_lds + (h_lds ? (size_t)P * 36 : 0);
    if (ckpt && (!aligned16(ckpt) || H < 2 || W < 2))
        return fail(MPIV_ERR_ARG, "%s: checkpoints must be 16-byte aligned (and come from mpiv_render_train)", nm);
    if (!aligned16(dmpi) || (reinterpret_cast<uintptr_t>(workspace) & 255))
        return fail(MPIV_ERR_ARG, "%s: d rgba_layers must be 16-byte and workspace 256-byte aligned", nm);
    // pixel ids, bucket ids and order keys are 32-bit
    if ((int64_t)H * W >= ((int64_t)1 << 26) || (int64_t)P * H * W >= ((int64_t)1 << 31))
        return fail(MPIV_ERR_ARG, "%s: MPI too large for one backward launch", nm);
    // plane groups: one (every plane's d samples resident) when the workspace holds it, else
    // groups of bwd_group_planes (mpiv_render_backward_workspace_size / _size_min)
    // Overlapped (round 5, default for views of more than one group): groups of bwd_group_planes in two
    // d-sample windows, group k's gather / check / fallback on a second stream while group k-1's chain
    // runs on the caller's (the chain is texture-path-bound, the gather latency-bound), when the
    // workspace holds two windows (the default workspace does)
    const bool fast2 = H >= 2 && W >= 2;
    const int GPo = bwd_group_planes(H, W, P);
    const bool overlap = MPIV_AB && opt(kOptBwdOverlap) != 0 && fast2 && GPo < P &&
                         ws_bytes >= bwd_layout(H, W, P, GPo, nullptr, nullptr, nullptr, 2);
    const int GP = overlap ? GPo : (opt(kOptBwdGroup) > 0 || ws_bytes < bwd_layout(H, W, P, P, nullptr, nullptr))
                                       ? bwd_group_planes(H, W, P) : P;
    const int G = (P + GP - 1) / GP;
    BwdWs ws, ws2;
    float4* gbuf = nullptr;
    const size_t need = bwd_layout(H, W, P, GP, static_cast<char*>(workspace), &ws, &gbuf, overlap ? 2 : 1, &ws2);
    if (ws_bytes < need) return fail(MPIV_ERR_ARG, "%s: workspace too small (%zu < %zu bytes)", nm, ws_bytes, need);
    const RenderGeom g = make_geom(H, W, P);
    const ChunkGeom cg{(int)(st[1] / 4), (int)(st[2] / 4), (int)rec};
    const bool fast = H >= 2 && W >= 2;
    const int64_t HW = (int64_t)H * W;
    {
        int d = 0;
        int* flags = watched && hipGetDevice(&d) == hipSuccess && d >= 0 && d < kAbortSlots ? abort_flags_dev() : nullptr;
        ws.sink = ws2.sink = flags ? flags + d : nullptr;
    }
    const int tiles_x = (int)blocks(W, kGTW);
    const int64_t ntiles = (int64_t)tiles_x * blocks(H, kGTY);
    const int64_t gather_blocks = ntiles * blocks(P, kGPl);
    if (gather_blocks > kMaxGridX) return fail(MPIV_ERR_ARG, "%s: too many blocks", nm);
    if (opt(kOptBwdGather) != 0 && !(MPIV_AB && MPIV_GTR == 1))
        return fail(MPIV_ERR_ARG, "%s: bwd_gather=%d needs an A/B build with one texel row per wave (-DMPIV_GTR=1)", nm,
                    opt(kOptBwdGather));
    const int force = opt(kOptBwdFallback) != 0 || !fast;
    const float margin = (float)opt(kOptBwdMargin) / 64.0f;
    hipStream_t q = S(stream);
    // fallback grid: at most the blocks that fit at once, <= 4 per CU (more would only wait for
    // tickets; fewer resident ones still complete); queried once per device (racing first calls
    // store the same values; the block count is published with release after the clock rate and
    // read with acquire, so a thread that sees it also sees the clock -- ADVICE r5)
    static int s_fb_blocks[64] = {};
    static long long s_clock_khz[64] = {};
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return fail(MPIV_ERR_HIP, "%s: hipGetDevice failed", nm);
    int fbb = __atomic_load_n(&s_fb_blocks[dev], __ATOMIC_ACQUIRE);
    if (fbb == 0) {
        int ncu = 0, pc_t = 0, pc_f = 0;
        if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
            hipOccupancyMaxActiveBlocksPerMultiprocessor(&pc_t, (const void*)bwd_fallback_kernel<true>, 256, 0) !=
                hipSuccess ||
            hipOccupancyMaxActiveBlocksPerMultiprocessor(&pc_f, (const void*)bwd_fallback_kernel<false>, 256, 0) !=
                hipSuccess ||
            ncu <= 0 || pc_t <= 0 || pc_f <= 0)
            return fail(MPIV_ERR_HIP, "%s: device query failed", nm);
        fbb = ncu * std::min(std::min(pc_t, pc_f), 4);
        int khz = 0;
        if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev) != hipSuccess || khz <= 0)
            khz = 100000;  // gfx9's constant 100 MHz wall clock
        __atomic_store_n(&s_clock_khz[dev], (long long)khz, __ATOMIC_RELAXED);
        __atomic_store_n(&s_fb_blocks[dev], fbb, __ATOMIC_RELEASE);
    }
    const unsigned fb_blocks = opt(kOptBwdFbBlocks) > 0 ? (unsigned)opt(kOptBwdFbBlocks) : (unsigned)fbb;
    const int pl = opt(kOptBwdPollLimit);
    // production: no poll-count limit, a 60 s wall-clock limit per wait (a poll budget
    // could expire on a slow but correct fallback); bwd_poll_limit=k (A/B, tests) adds a count limit
    const unsigned poll_limit = pl > 0 ? (unsigned)pl : pl < 0 ? 0u : ~0u;
    const long long khz_seen = __atomic_load_n(&s_clock_khz[dev], __ATOMIC_RELAXED);
    const unsigned long long tick_limit = 60000ull * (unsigned long long)(khz_seen > 0 ? khz_seen : 100000);
    const int fb_mode = opt(kOptBwdFbMode);
    // Launch-folded schedule (round 6; one plane group, tile gather): per view the box kernel (the planes'
    // inverses inside, and block 0 zeroing the counters this memset would) runs first, the pair-count
    // check runs in the gather's last block and the NaN fill of an aborted view in the fallback's last
    // block: 4 launches per view instead of 7 plus the memset (the notebook's 224x224 training step is
    // launch-bound).  The other schedules keep the separate launches.
    const bool folded = !force && G == 1 && !overlap && opt(kOptBwdUnfold) == 0 && opt(kOptBwdGather) == 0 && fb_mode != 1;
    // truth, found, flag (adjacent), and the second window's set after them
    if (!folded &&
        hipMemsetAsync(ws.truth, 0, overlap ? 2 * (2 * kCtrSlots * 8 + 256) : 2 * kCtrSlots * 8 + 256, q) != hipSuccess)
        return fail(MPIV_ERR_HIP, "%s: hipMemsetAsync failed", nm);
    if (overlap) {
        std::lock_guard<std::mutex> lk(g_aux_mu);
        BwdAux* ax = bwd_aux(dev);
        if (ax) {
            hipStream_t a = ax->s;
            bool ok = true;
            auto chk = [&](hipError_t e) { ok = ok && e == hipSuccess; };
            BwdWs win[2] = {ws, ws2};
            win[0].vcount = win[1].vcount = nullptr;  // bwd_poison_kernel counts the aborted views
            for (int v = 0; v < V && ok; ++v) {
                const float* hv = homs + (int64_t)v * P * 9;
                const float* dv = dout + (int64_t)v * HW * 3;
                const float* mv = mpi + (int64_t)v * st[0];
                float4* gv = reinterpret_cast<float4*>(dmpi) + (int64_t)v * HW * P;
                const float4* ckv = ckpt ? reinterpret_cast<const float4*>(ckpt) +
                                               (int64_t)v * ((P + kBwdCH - 1) / kBwdCH) * HW
                                         : nullptr;
                // the previous view's second-stream work (it reads ws.box / ws.inv and both windows)
                if (v > 0) chk(hipStreamWaitEvent(q, ax->view, 0));
                if (!ckv) {  // the checkpoints from a forward pass into the workspace (frame into gbuf, unused)
                    const unsigned fb = blocks(W, kStripTX) * blocks(H, 16);
                    const size_t flds = (size_t)chunk_slot_floats<8, 1>() * 4 + (h_lds ? (size_t)P * 36 : 0);
                    render_chunk_strip_kernel<16, 2><<<fb, 256, flds, q>>>(mv, 0, g, cg, 1, hv,
                                                                          reinterpret_cast<float*>(gbuf), ws.ckpt, h_lds);
                    ckv = ws.ckpt;
                }
                if (!force)  // the planes' inverses computed inside (one launch fewer)
                    bwd_box_kernel<true><<<blocks((int64_t)P * ntiles, 256), 256, 0, q>>>(
                        g, hv, ws.inv, (int)ntiles, tiles_x, margin, ws.box, (double)W / (H - 1), (double)H / (W - 1));
                for (int grp = G - 1; grp >= 0 && ok; --grp) {
                    const int k = G - 1 - grp, par = k & 1;
                    const int p_lo = grp * GP, p_hi = std::min(P, p_lo + GP);
                    if (k >= 2) chk(hipStreamWaitEvent(q, ax->done[par], 0));  // window par is free again
                    BwdWs wg = win[par];
                    wg.ds_p0 = p_lo;  // the window holds the group's d samples: planes p_lo .. p_hi-1
                    bwd_chain_strip_kernel<8><<<blocks(W, kStripTX) * blocks(H, 8), 256, chain_lds, q>>>(
                        mv, g, cg, hv, dv, ckv, wg, h_lds, p_lo / kBwdCH, (p_hi + kBwdCH - 1) / kBwdCH, gbuf);
                    chk(hipEventRecord(ax->chain[par], q));
                    chk(hipStreamWaitEvent(a, ax->chain[par], 0));
                    if (!force)
                        bwd_gather_kernel<false><<<(unsigned)(ntiles * blocks(p_hi - p_lo, kGPl)), kGThreads, 0, a>>>(
                            g, hv, wg, gv, margin, p_lo, p_hi - p_lo);
                    bwd_check_kernel<<<1, kWave, 0, a>>>(wg, force, k >= 2);
                    bwd_fallback_kernel<true><<<fb_blocks, 256, 0, a>>>(g, hv, wg, gv, poll_limit, tick_limit,
                                                                        fb_mode == 2, p_lo, p_hi);
                    chk(hipEventRecord(ax->done[par], a));
                }
                // an aborted group (never expected) leaves the view's gradient NaN, counted once
                bwd_poison_kernel<<<256, 256, 0, a>>>(win[0].flag, gv, (int64_t)P * HW, win[1].flag, ws.flag + 4, ws.sink);
                chk(hipEventRecord(ax->view, a));
            }
            chk(hipStreamWaitEvent(q, ax->view, 0));  // the caller's stream: every launch of this call
            if (!ok) return fail(MPIV_ERR_HIP, "%s: stream event failed", nm);
            return launched(nm);
        }
        // no second stream: the sequential schedule below on the first window
    }
    for (int v = 0; v < V; ++v) {
        const float* hv = homs + (int64_t)v * P * 9;
        const float* dv = dout + (int64_t)v * HW * 3;
        const float* mv = mpi + (int64_t)v * st[0];
        float4* gv = reinterpret_cast<float4*>(dmpi) + (int64_t)v * HW * P;
        const float4* ck = ckpt ? reinterpret_cast<const float4*>(ckpt) + (int64_t)v * ((P + kBwdCH - 1) / kBwdCH) * HW
                                : nullptr;
        if (G > 1) {  // several plane groups, back to front (fast recipe: H, W >= 2 here, P * H * W > 2^25)
            const float4* ckv = ck;
            if (!ckv) {  // the checkpoints from a forward pass into the workspace (frame into gbuf, unused)
                const unsigned fb = blocks(W, kStripTX) * blocks(H, 16);
                const size_t flds = (size_t)chunk_slot_floats<8, 1>() * 4 + (h_lds ? (size_t)P * 36 : 0);
                render_chunk_strip_kernel<16, 2><<<fb, 256, flds, q>>>(mv, 0, g, cg, 1, hv, reinterpret_cast<float*>(gbuf),
                                                                      ws.ckpt, h_lds);
                ckv = ws.ckpt;
            }
            if (!force)  // the planes' inverses computed inside (one launch fewer)
                bwd_box_kernel<true><<<blocks((int64_t)P * ntiles, 256), 256, 0, q>>>(
                    g, hv, ws.inv, (int)ntiles, tiles_x, margin, ws.box, (double)W / (H - 1), (double)H / (W - 1));
            for (int grp = G - 1; grp >= 0; --grp) {
                const int p_lo = grp * GP, p_hi = std::min(P, p_lo + GP);
                BwdWs wg = ws;
                wg.ds_p0 = p_lo;  // the window holds the group's d samples: planes p_lo .. p_hi-1
                bwd_chain_strip_kernel<8><<<blocks(W, kStripTX) * blocks(H, 8), 256, chain_lds, q>>>(
                    mv, g, cg, hv, dv, ckv, wg, h_lds, p_lo / kBwdCH, (p_hi + kBwdCH - 1) / kBwdCH, gbuf);
                if (!force)
                    bwd_gather_kernel<false><<<(unsigned)(ntiles * blocks(p_hi - p_lo, kGPl)), kGThreads, 0, q>>>(
                        g, hv, wg, gv, margin, p_lo, p_hi - p_lo);
                bwd_check_kernel<<<1, kWave, 0, q>>>(wg, force, grp != G - 1);
                if (fast)
                    bwd_fallback_kernel<true><<<fb_blocks, 256, 0, q>>>(g, hv, wg, gv, poll_limit, tick_limit, fb_mode == 2, p_lo,
                                                                        p_hi);
                else
                    bwd_fallback_kernel<false><<<fb_blocks, 256, 0, q>>>(g, hv, wg, gv, poll_limit, tick_limit, fb_mode == 2, p_lo,
                                                                         p_hi);
            }
            bwd_poison_kernel<<<256, 256, 0, q>>>(ws.flag, gv, (int64_t)P * HW, nullptr, nullptr, ws.sink);
            continue;
        }
        const int R = fast ? chunk_rows() : 1;
        const unsigned cb = blocks(W, kTileX) * blocks(H, kTileY * R);
        if (folded)  // the boxes (and the planes' inverses) first; block 0 zeroes the counters
            bwd_box_kernel<true><<<blocks((int64_t)P * ntiles, 256), 256, 0, q>>>(
                g, hv, ws.inv, (int)ntiles, tiles_x, margin, ws.box, (double)W / (H - 1), (double)H / (W - 1), ws,
                v == 0 ? 2 : 1);
        if (!ck && fast && R == 1 && opt(kOptChunkStrip) == 1) {
            // no checkpoints: a strip forward pass writes them into the workspace (its frame into
            // this view's d MPI, which the gather / fallback overwrite), then the one-pass chain --
            // 0.6 + 2.4 ms against 3.0-3.1 for the two-pass chain
            const unsigned fb = blocks(W, kStripTX) * blocks(H, 16);
            const size_t flds = (size_t)chunk_slot_floats<8, 1>() * 4 + (h_lds ? (size_t)P * 36 : 0);
            render_chunk_strip_kernel<16, 2><<<fb, 256, flds, q>>>(mv, 0, g, cg, 1, hv, reinterpret_cast<float*>(gv),
                                                                  ws.ckpt, h_lds);
            ck = ws.ckpt;
        }
#define MPIV_CHAIN(CKB, RR)                                                                                  \
    bwd_chain_kernel<1, CKB, RR><<<cb, 256, chain_lds, q>>>(mv, g, cg, hv, dv, CKB ? ck : nullptr, ws, h_lds)
        if (!fast)
            bwd_chain_kernel<0, false, 1><<<cb, 256, chain_lds, q>>>(mv, g, cg, hv, dv, nullptr, ws, h_lds);
#if MPIV_AB  // R rows per wave: measured slower
        else if (ck && R == 4) MPIV_CHAIN(true, 4);
        else if (ck && R == 2) MPIV_CHAIN(true, 2);
        else if (!ck && R == 4) MPIV_CHAIN(false, 4);
        else if (!ck && R == 2) MPIV_CHAIN(false, 2);
#endif
#if MPIV_AB
        else if (ck && opt(kOptChunkStrip) == 4)  // A/B: 8 x 16 strips (2.41 vs 2.38 ms, r04j_strips_ab.jsonl)
            bwd_chain_strip_kernel<16><<<blocks(W, kStripTX) * blocks(H, 16), 256, chain_lds, q>>>(mv, g, cg, hv, dv, ck,
                                                                                                ws, h_lds, 0, (P + 7) / 8,
                                                                                                gbuf);
#endif
        else if (ck && opt(kOptChunkStrip))  // 8 x 8 strips, vertical tap reuse
            bwd_chain_strip_kernel<8><<<blocks(W, kStripTX) * blocks(H, 8), 256, chain_lds, q>>>(mv, g, cg, hv, dv, ck,
                                                                                              ws, h_lds, 0, (P + 7) / 8,
                                                                                              gbuf);
        else if (ck) MPIV_CHAIN(true, 1);
        else MPIV_CHAIN(false, 1);
#undef MPIV_CHAIN
        if (folded) {
            // the check in the gather's last block costs every block a wait for its stores and a barrier at
            // its end (+2 % at config 4's 131072 blocks, profiles/r06_bwd_fold.json): small grids only, where
            // the separate launch is what costs
            if (gather_blocks <= kFoldCheckMaxBlocks) {
                bwd_gather_kernel<true><<<(unsigned)gather_blocks, kGThreads, 0, q>>>(g, hv, ws, gv, margin, 0, P);
            } else {
                bwd_gather_kernel<false><<<(unsigned)gather_blocks, kGThreads, 0, q>>>(g, hv, ws, gv, margin, 0, P);
                bwd_check_kernel<<<1, kWave, 0, q>>>(ws, 0, 0);
            }
            if (fast)
                bwd_fallback_kernel<true><<<fb_blocks, 256, 0, q>>>(g, hv, ws, gv, poll_limit, tick_limit, fb_mode == 2, 0,
                                                                    P, (int64_t)P * HW);
            else
                bwd_fallback_kernel<false><<<fb_blocks, 256, 0, q>>>(g, hv, ws, gv, poll_limit, tick_limit, fb_mode == 2, 0,
                                                                     P, (int64_t)P * HW);
            continue;
        }
        if (!force) {
#if MPIV_AB && MPIV_GTR == 1  // one texel row per wave / staging and texel waves: measured slower
            if (opt(kOptBwdGather) == 1) {
                bwd_inverse_kernel<<<blocks(P, 64), 64, 0, q>>>(hv, P, (double)W / (H - 1), (double)H / (W - 1), ws.inv);
                bwd_gather_wave_kernel<<<(unsigned)gather_blocks, 256, 0, q>>>(g, hv, ws, gv, margin);
            } else
#endif
            {
                // the planes' inverses computed inside (bwd_plane_inverse, the same floats): one launch fewer
                bwd_box_kernel<true><<<blocks((int64_t)P * ntiles, 256), 256, 0, q>>>(
                    g, hv, ws.inv, (int)ntiles, tiles_x, margin, ws.box, (double)W / (H - 1), (double)H / (W - 1));
#if MPIV_AB && MPIV_GTR == 1
                if (opt(kOptBwdGather) == 2)
                    bwd_gather_ws_kernel<<<(unsigned)gather_blocks, 2 * kGThreads, 0, q>>>(g, hv, ws, gv, margin);
                else if (opt(kOptBwdGather) == 3)
                    bwd_gather_dma_kernel<<<(unsigned)gather_blocks, kGThreads, 0, q>>>(g, hv, ws, gv, margin);
                else
#endif
                    bwd_gather_kernel<false><<<(unsigned)gather_blocks, kGThreads, 0, q>>>(g, hv, ws, gv, margin, 0, P);
            }
        }
        bwd_check_kernel<<<1, kWave, 0, q>>>(ws, force, 0);
        // fallback: one launch, returns at once unless flagged; its phases are ordered by tickets
        // (render_bwd.hip), so it completes however many of its blocks are resident
#if MPIV_AB  // round 3's grid-barrier schedule (render_bwd.hip; it needs every block resident, so it
            // keeps its poll-count limit)
        const unsigned bar_polls = poll_limit == ~0u ? (1u << 24) : poll_limit;
        if (fb_mode == 1 && fast)
            bwd_fallback_barrier_kernel<true><<<fb_blocks, 256, 0, q>>>(g, hv, ws, gv, bar_polls);
        else if (fb_mode == 1)
            bwd_fallback_barrier_kernel<false><<<fb_blocks, 256, 0, q>>>(g, hv, ws, gv, bar_polls);
        else
#endif
        if (fast)
            bwd_fallback_kernel<true><<<fb_blocks, 256, 0, q>>>(g, hv, ws, gv, poll_limit, tick_limit, fb_mode == 2, 0, P);
        else
            bwd_fallback_kernel<false><<<fb_blocks, 256, 0, q>>>(g, hv, ws, gv, poll_limit, tick_limit, fb_mode == 2, 0, P);
        // an aborted fallback (never expected) leaves a NaN gradient, never a plausible one
        bwd_poison_kernel<<<256, 256, 0, q>>>(ws.flag, gv, (int64_t)P * HW, nullptr, nullptr, ws.sink);
    }
    return launched(nm);
}

int mpiv_render_backward(const float* mpi, const int64_t st[5], int V, int H, int W, int P, const float* homs,
                         const float* dout, const float* ckpt, float* dmpi, void* workspace, size_t ws_bytes,
                         void* stream) {
    return render_backward_impl("mpiv_render_backward", mpi, st, V, H, W, P, homs, dout, ckpt, dmpi, workspace, ws_bytes,
                                stream, false);
}

int mpiv_render_backward_watched(const float* mpi, const int64_t st[5], int V, int H, int W, int P, const float* homs,
                                 const float* dout, const float* ckpt, float* dmpi, void* workspace, size_t ws_bytes,
                                 void* stream) {
    if (!abort_flags_dev()) return fail(MPIV_ERR_HIP, "mpiv_render_backward_watched: no page-locked abort flag");
    return render_backward_impl("mpiv_render_backward_watched", mpi, st, V, H, W, P, homs, dout, ckpt, dmpi, workspace,
                                ws_bytes, stream, true);
}

int mpiv_render_backward_status(const void* workspace, int H, int W, int P, int* aborted_views, void* stream) {
    const char* nm = "mpiv_render_backward_status";
    if (!workspace || !aborted_views) return fail(MPIV_ERR_ARG, "%s: null pointer", nm);
    if (H <= 0 || W <= 0 || P <= 0) return fail(MPIV_ERR_ARG, "%s: bad shape", nm);
    BwdWs ws;  // (the flag words sit at the same offset for every group size)
    bwd_layout(H, W, P, P, static_cast<char*>(const_cast<void*>(workspace)), &ws);
    hipStream_t q = S(stream);
    if (hipMemcpyAsync(aborted_views, ws.flag + 4, sizeof(int), hipMemcpyDeviceToHost, q) != hipSuccess ||
        hipStreamSynchronize(q) != hipSuccess)
        return fail(MPIV_ERR_HIP, "%s: copy failed", nm);
    g_err[0] = '\0';
    return MPIV_OK;
}

int mpiv_combine_ct(const float* parts, int G, int64_t n, float* out, void* stream) {
    if (!parts || !out) return fail(MPIV_ERR_ARG, "mpiv_combine_ct: null pointer");
    if (G <= 0 || n <= 0) return fail(MPIV_ERR_ARG, "mpiv_combine_ct: bad shape");
    if (!aligned16(parts)) return fail(MPIV_ERR_ARG, "mpiv_combine_ct: parts must be 16-byte aligned");
    combine_ct_kernel<<<blocks(n, 256), 256, 0, S(stream)>>>(reinterpret_cast<const float4*>(parts), n, G, n, out);
    return launched("mpiv_combine_ct");
}

static SweepParams sweep_params(int B, int Hs, int Ws, int C, int D, int Ht, int Wt) {
    SweepParams sp;
    sp.B = B; sp.Hs = Hs; sp.Ws = Ws; sp.C = C; sp.D = D; sp.Ht = Ht; sp.Wt = Wt;
    sp.fhs = (float)Hs;
    sp.fws = (float)Ws;
    sp.half_ws = (float)Ws * 0.5f;
    sp.half_hs = (float)Hs * 0.5f;
    return sp;
}

#if MPIV_AB
// blocks of plane_sweep_pf_kernel resident at once (CUs x blocks per CU), queried once per device;
// a dry run without a device reports MI355X's 256 CUs x 3
static int sweep_pf_blocks() {
    static int s_blocks[64] = {};
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return g_route ? 256 * 3 : 0;
    int nb = __atomic_load_n(&s_blocks[dev], __ATOMIC_RELAXED);
    if (nb == 0) {
        int ncu = 0, per = 0;
        if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
            hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, (const void*)plane_sweep_pf_kernel<3, 1>, kDLThreads, 0) !=
                hipSuccess ||
            ncu <= 0 || per <= 0)
            return g_route ? 256 * 3 : 0;
        nb = ncu * per;
        __atomic_store_n(&s_blocks[dev], nb, __ATOMIC_RELAXED);
    }
    return nb;
}
#endif

// plane_sweep_dlane_kernel on the caller's strided source (C <= 4): no padded copy
static int sweep_raw_into(const char* nm, const float* img, const int64_t st[4], int B, int Hs, int Ws, int C,
                          const float* ki, const float* proj, const float* depths, int D, int Ht, int Wt, float* out,
                          int64_t out_bstride, int64_t out_pstride, void* stream) {
    if (out_pstride < (int64_t)D * C || out_pstride > (1 << 30) || out_bstride < (int64_t)Ht * Wt * out_pstride ||
        (int64_t)Ht * Wt >= (1ll << 31))
        return fail(MPIV_ERR_ARG, "%s: bad output strides", nm);
    if (Hs >= (1 << 22) || Ws >= (1 << 22)) return fail(MPIV_ERR_ARG, "%s: a source side >= 2^22", nm);
    // tile rows: sweep_rows option, else 4 (automatic)
    const int so = opt(kOptSweepRows);
    const int SLR = (so == 6 || so == 8) ? so : 4;
    const int64_t tiles = (int64_t)((Wt + kSLP - 1) / kSLP) * ((Ht + SLR - 1) / SLR);
    if (B > kMaxGridYZ || tiles > kMaxGridX) return fail(MPIV_ERR_ARG, "%s: too large", nm);
    const SweepParams sp = sweep_params(B, Hs, Ws, C, D, Ht, Wt);
    const float rc_hs = 1.0f / sp.fhs, rc_ws = 1.0f / sp.fws;
    const ImgStrides is{st[0], st[1], st[2], st[3]};
    const bool vec = aligned16(out) && out_pstride % 4 == 0 && out_bstride % 4 == 0;
    const dim3 lgrid((unsigned)tiles, B, 1);
    const int shrink = opt(kOptBoxShrink);
    hipStream_t q = S(stream);
    // few depths: no LDS staging (plane_sweep_direct_kernel); sweep_direct = -1 off, 1 for any D <= 64
    const int od = opt(kOptSweepDirect);
    // automatic: D <= 2 direct, 3 <= D <= 8 pixel per lane, deeper the LDS-staged kernel
    // (profiles/r03_sweep_few_depths_ab.txt)
    const bool px_auto = od == 0 && D >= 3 && D <= kDirMaxD;
    if ((px_auto || od == 2 || od == 3) && D * C <= kPxMaxDC && shrink == 0 && Ht <= (int)kMaxGridYZ) {
        // pixel per lane, the wave's samples staged in LDS and stored as one run
        // (plane_sweep_px_kernel; 64 pixels per wave, 32 with sweep_direct=3)
        const int PW = od == 3 ? kWave / 2 : kWave;
        const dim3 pgrid((unsigned)((Wt + 4 * PW - 1) / (4 * PW)), (unsigned)Ht, (unsigned)B);
        const int CC = C < 4 ? C : 4;
        const size_t lds = (size_t)4 * PW * D * CC * sizeof(float);
        if (g_route) return note_route((int64_t)pgrid.x * Ht * B, 256, "plane_sweep_px_kernel<%d, %d>", CC, PW);
        const float rDC = 1.0f / (float)(D * CC);
#define MPIV_PX1(K, PP)                                                                                    \
    plane_sweep_px_kernel<K, PP><<<pgrid, 256, lds, q>>>(img, is, sp, rc_hs, rc_ws, rDC, ki, proj, depths, \
                                                         out, out_bstride, out_pstride, (int)vec)
#define MPIV_PX(K)                     \
    if (PW == kWave) MPIV_PX1(K, kWave); \
    else MPIV_PX1(K, kWave / 2)
        switch (C) {
            case 1: MPIV_PX(1); break;
            case 2: MPIV_PX(2); break;
            case 3: MPIV_PX(3); break;
            default: MPIV_PX(4); break;
        }
#undef MPIV_PX
#undef MPIV_PX1
        return launched(nm);
    }
    if (od >= 0 && od < 2 && shrink == 0 && D <= (od == 1 ? kWave : kDirMaxD) && Ht <= (int)kMaxGridYZ) {
        const int ppw = kWave / D;
        const int64_t gpr = (Wt + ppw - 1) / ppw;  // pixel groups per target row
        const dim3 dgrid((unsigned)((gpr + 4 * kDirG - 1) / (4 * kDirG)), (unsigned)Ht, (unsigned)B);
        if (g_route) return note_route((int64_t)dgrid.x * Ht * B, 256, "plane_sweep_direct_kernel<%d>", C < 4 ? C : 4);
        const float rD = 1.0f / (float)D;
#define MPIV_DIRECT(CC)                                                                                      \
    plane_sweep_direct_kernel<CC><<<dgrid, 256, 0, q>>>(img, is, sp, rc_hs, rc_ws, rD, ki, proj, depths, out, \
                                                        out_bstride, out_pstride, (int)vec)
        switch (C) {
            case 1: MPIV_DIRECT(1); break;
            case 2: MPIV_DIRECT(2); break;
            case 3: MPIV_DIRECT(3); break;
            default: MPIV_DIRECT(4); break;
        }
#undef MPIV_DIRECT
        return launched(nm);
    }
    // persistent tiles with the next tile's box and texels prefetched (plane_sweep_pf_kernel)
    const int opf = opt(kOptSweepPf);
    (void)opf;
    // (fills through a buffer resource over each source image: non-negative strides, a span under 2 GiB)
    const int64_t span = ((int64_t)(Hs - 1) * st[1] + (int64_t)(Ws - 1) * st[2] + (int64_t)(C - 1) * st[3] + 1) * 4;
    const bool rs_ok = st[1] >= 0 && st[2] >= 0 && st[3] >= 0 && st[1] < (1 << 28) && st[2] < (1 << 28) &&
                       st[3] < (1 << 28) && span < kOOB - 64;
    [[maybe_unused]] const bool pf_ok = rs_ok && tiles * B < (1ll << 31);
    const int span32 = rs_ok ? (int)span : 0;  // the staged kernels' buffer-resource fill (0: masked pointer loads)
#if MPIV_AB  // measured slower than one block per tile
    if (SLR == 4 && shrink == 0 && pf_ok && opt(kOptSweepBand) == 0 && opf > 0) {
        const int64_t total = tiles * B;
        const int res = sweep_pf_blocks();
        if (res <= 0) return fail(MPIV_ERR_HIP, "%s: device query failed", nm);
        const unsigned G = (unsigned)std::min<int64_t>(total, res);
        if (g_route) return note_route(G, kDLThreads, "plane_sweep_pf_kernel<%d, 1>", C < 4 ? C : 4);
#define MPIV_PF(CC)                                                                                             \
    plane_sweep_pf_kernel<CC, 1><<<G, kDLThreads, 0, q>>>(img, st[0], (int)st[1], (int)st[2], (int)st[3], sp,    \
                                                          rc_hs, rc_ws, ki, proj, depths, out,                    \
                                                          out_bstride, out_pstride, (int)vec, shrink, (int)tiles, \
                                                          (int)total, (int)span)
        switch (C) {
            case 1: MPIV_PF(1); break;
            case 2: MPIV_PF(2); break;
            case 3: MPIV_PF(3); break;
            default: MPIV_PF(4); break;
        }
#undef MPIV_PF
        return launched(nm);
    }
#endif
    // one pixel per lane and iteration for few depths (D = 10: 0.228 vs 0.243 ms), two above
    // (D = 64: 0.640 vs 0.652; profiles/r03_sweep_few_depths_ab.txt)
    const int pix = (SLR == 4 && D <= 16) ? 1 : kDLPix;
    const bool soa = MPIV_AB && opt(kOptSweepSoa) > 0;
    if (g_route && !(MPIV_AB && opt(kOptSweepBand) != 0 && SLR == 4))
        return note_route(tiles * B, kDLThreads, "plane_sweep_dlane_kernel<%d, true, %d, %d, %d, %s>", C < 4 ? C : 4, SLR,
                          SLR == 4 ? kSLCap : 4096, pix, soa ? "true" : "false");  // (rocprof prints every argument)
#define MPIV_DLRAW1(CC, RR, CAP, PP, SO)                                                                           \
    plane_sweep_dlane_kernel<CC, true, RR, CAP, PP, SO><<<lgrid, kDLThreads, 0, q>>>(nullptr, PadGeom{0, 0, 0, 0}, img, \
                                                                                    is, sp, rc_hs, rc_ws, ki, proj,     \
                                                                                    depths, out, out_bstride,           \
                                                                                    out_pstride, (int)vec, shrink, span32)
#if MPIV_AB  // channel-planar staging: measured slower
#define MPIV_DLRAW(CC, RR, CAP, PP)         \
    if (soa) MPIV_DLRAW1(CC, RR, CAP, PP, true); \
    else MPIV_DLRAW1(CC, RR, CAP, PP, false)
#else
#define MPIV_DLRAW(CC, RR, CAP, PP) MPIV_DLRAW1(CC, RR, CAP, PP, false)
#endif
#define MPIV_DLRAW_C(RR, CAP, PP)                  \
    switch (C) {                                   \
        case 1: MPIV_DLRAW(1, RR, CAP, PP); break; \
        case 2: MPIV_DLRAW(2, RR, CAP, PP); break; \
        case 3: MPIV_DLRAW(3, RR, CAP, PP); break; \
        default: MPIV_DLRAW(4, RR, CAP, PP); break; \
    }
#if MPIV_AB  // taller tiles: measured within noise
    if (SLR == 8) {
        MPIV_DLRAW_C(8, 4096, kDLPix)
    } else if (SLR == 6) {
        MPIV_DLRAW_C(6, 4096, kDLPix)
    } else
#endif
#if MPIV_AB  // the band-walking ring kernel: measured slower than one box per tile
    if (opt(kOptSweepBand) != 0 && SLR == 4) {
        // band-walking kernel (round 5): bands of kBandSteps 4-row tiles, source rows in an LDS ring
        const int64_t bands = (int64_t)((Wt + kSLP - 1) / kSLP) * ((Ht + 4 * kBandSteps - 1) / (4 * kBandSteps));
        const dim3 bgrid((unsigned)bands, B, 1);
        if (g_route) return note_route(bands * B, kDLThreads, "plane_sweep_band_kernel<%d, %d>", C < 4 ? C : 4, pix);
#define MPIV_BAND(CC, PP)                                                                                   \
    plane_sweep_band_kernel<CC, PP><<<bgrid, kDLThreads, 0, q>>>(img, is, sp, rc_hs, rc_ws, ki, proj, depths, out, \
                                                                out_bstride, out_pstride, (int)vec, shrink)
#define MPIV_BAND_C(PP)                    \
    switch (C) {                           \
        case 1: MPIV_BAND(1, PP); break;   \
        case 2: MPIV_BAND(2, PP); break;   \
        case 3: MPIV_BAND(3, PP); break;   \
        default: MPIV_BAND(4, PP); break;  \
    }
        if (pix == 1) {
            MPIV_BAND_C(1)
        } else {
            MPIV_BAND_C(kDLPix)
        }
#undef MPIV_BAND_C
#undef MPIV_BAND
    } else
#endif
    if (pix == 1) {
        MPIV_DLRAW_C(4, kSLCap, 1)
    } else {
        MPIV_DLRAW_C(4, kSLCap, kDLPix)
    }
#undef MPIV_DLRAW_C
#undef MPIV_DLRAW
#undef MPIV_DLRAW1
    return launched(nm);
}

int mpiv_plane_sweep_into(const float* img, const int64_t st[4], int B, int Hs, int Ws, int C, const float* ki,
                          const float* proj, const float* depths, int D, int Ht, int Wt, float* out,
                          int64_t out_bstride, int64_t out_pstride, void* stream) {
    if (!img || !st || !ki || !proj || !depths || !out)
        return fail(MPIV_ERR_ARG, "mpiv_plane_sweep_into: null pointer");
    if (B <= 0 || Hs <= 0 || Ws <= 0 || C <= 0 || C > 4 || D <= 0 || Ht <= 0 || Wt <= 0)
        return fail(MPIV_ERR_ARG, "mpiv_plane_sweep_into: bad shape");
    return sweep_raw_into("mpiv_plane_sweep_into", img, st, B, Hs, Ws, C, ki, proj, depths, D, Ht, Wt, out,
                          out_bstride, out_pstride, stream);
}

int mpiv_plane_sweep(const float* img, const int64_t st[4], int B, int Hs, int Ws, int C, const float* ki,
                     const float* proj, const float* depths, int D, int Ht, int Wt, float* out, void* stream) {
    if (!img || !st || !ki || !proj || !depths || !out) return fail(MPIV_ERR_ARG, "mpiv_plane_sweep: null pointer");
    if (B <= 0 || Hs <= 0 || Ws <= 0 || C <= 0 || D <= 0 || Ht <= 0 || Wt <= 0)
        return fail(MPIV_ERR_ARG, "mpiv_plane_sweep: bad shape");
    // C <= 4: the depth-per-lane LDS kernel reading the source in place (sweep_dlane=0: the
    // generic one-sample-per-thread kernel, as for C > 4)
    if (C <= 4 && opt(kOptSweepDlane) != 0)
        return sweep_raw_into("mpiv_plane_sweep", img, st, B, Hs, Ws, C, ki, proj, depths, D, Ht, Wt, out,
                              (int64_t)Ht * Wt * D * C, (int64_t)D * C, stream);
    const int64_t per_view = (int64_t)Ht * Wt * D;
    if (B > kMaxGridYZ || blocks(per_view, 256) > kMaxGridX) return fail(MPIV_ERR_ARG, "mpiv_plane_sweep: too large");
    const ImgStrides s{st[0], st[1], st[2], st[3]};
    dim3 grid(blocks(per_view, 256), B, 1);
    if (g_route) return note_route((int64_t)grid.x * B, 256, "plane_sweep_kernel");
    plane_sweep_kernel<<<grid, 256, 0, S(stream)>>>(img, s, sweep_params(B, Hs, Ws, C, D, Ht, Wt), ki, proj, depths,
                                                    out);
    return launched("mpiv_plane_sweep");
}

// mpiv_plane_sweep for a pose already in HBM: proj = [[K_src, 0], [0, 0, 0, 1]] @ pose formed on
// the device into proj_scratch (mpiv_psv_proj_device's kernel) and the sweep, one call.
int mpiv_plane_sweep_pose(const float* img, const int64_t st[4], int B, int Hs, int Ws, int C, const float* ki,
                          const float* Ks, int64_t ks_bstride, const float* pose, float* proj_scratch,
                          const float* depths, int D, int Ht, int Wt, float* out, void* stream) {
    const char* nm = "mpiv_plane_sweep_pose";
    if (!Ks || !pose || !proj_scratch) return fail(MPIV_ERR_ARG, "%s: null pointer", nm);
    if (B <= 0 || ks_bstride < 0) return fail(MPIV_ERR_ARG, "%s: bad shape", nm);
    if (g_route) return mpiv_plane_sweep(img, st, B, Hs, Ws, C, ki, proj_scratch, depths, D, Ht, Wt, out, stream);
    psv_proj_kernel<<<blocks(B, 64), 64, 0, S(stream)>>>(Ks, ks_bstride, pose, B, proj_scratch);
    if (int rc = launched(nm)) return rc;
    return mpiv_plane_sweep(img, st, B, Hs, Ws, C, ki, proj_scratch, depths, D, Ht, Wt, out, stream);
}

int mpiv_pad_texels(const float* img, const int64_t st[4], int B, int Hs, int Ws, int C, float* img4,
                    void* stream) {
    if (!img || !st || !img4) return fail(MPIV_ERR_ARG, "mpiv_pad_texels: null pointer");
    if (B <= 0 || Hs <= 0 || Ws <= 0 || C <= 0 || C > 4) return fail(MPIV_ERR_ARG, "mpiv_pad_texels: bad shape");
    if (!aligned16(img4)) return fail(MPIV_ERR_ARG, "mpiv_pad_texels: img4 must be 16-byte aligned");
    if ((int64_t)(Hs + 2 * kPad) * (Ws + 2 * kPad) * 16 >= (int64_t)kOOB)
        return fail(MPIV_ERR_ARG, "mpiv_pad_texels: padded image larger than 2 GiB");
    if (B > kMaxGridYZ) return fail(MPIV_ERR_ARG, "mpiv_pad_texels: too large");
    const ImgStrides s{st[0], st[1], st[2], st[3]};
    const int64_t npix = (int64_t)(Hs + 2 * kPad) * (Ws + 2 * kPad);
    pad_texels_kernel<<<dim3(blocks(npix, 256), B), 256, 0, S(stream)>>>(
        img, s, Hs, Ws, C, make_fastdiv((unsigned)(Ws + 2 * kPad)), reinterpret_cast<float4*>(img4));
    return launched("mpiv_pad_texels");
}

int mpiv_plane_sweep_padded_into(const float* img4, int B, int Hs, int Ws, int C, const float* ki,
                                 const float* proj, const float* depths, int D, int Ht, int Wt, float* out,
                                 int64_t out_bstride, int64_t out_pstride, void* stream) {
    if (!img4 || !ki || !proj || !depths || !out) return fail(MPIV_ERR_ARG, "mpiv_plane_sweep_padded: null pointer");
    if (B <= 0 || Hs <= 0 || Ws <= 0 || C <= 0 || C > 4 || D <= 0 || Ht <= 0 || Wt <= 0)
        return fail(MPIV_ERR_ARG, "mpiv_plane_sweep_padded: bad shape");
    if (!aligned16(img4)) return fail(MPIV_ERR_ARG, "mpiv_plane_sweep_padded: img4 must be 16-byte aligned");
    if (out_pstride < (int64_t)D * C || out_pstride > (1 << 30) || out_bstride < (int64_t)Ht * Wt * out_pstride ||
        (int64_t)Ht * Wt >= (1ll << 31))
        return fail(MPIV_ERR_ARG, "mpiv_plane_sweep_padded: bad output strides");
    if ((int64_t)(Hs + 2 * kPad) * (Ws + 2 * kPad) * 16 >= (int64_t)kOOB || Hs >= (1 << 22) || Ws >= (1 << 22))
        return fail(MPIV_ERR_ARG, "mpiv_plane_sweep_padded: padded image > 2 GiB or a side >= 2^22");
    const int NG = (D + kSweepDG - 1) / kSweepDG;
    const int64_t per_view = (int64_t)Ht * Wt * NG;
    if (B > kMaxGridYZ || per_view >= (1ll << 31)) return fail(MPIV_ERR_ARG, "mpiv_plane_sweep_padded: too large");
    [[maybe_unused]] const FastDiv fd_g = make_fastdiv((unsigned)NG), fd_w = make_fastdiv((unsigned)Wt);
    const SweepParams sp = sweep_params(B, Hs, Ws, C, D, Ht, Wt);
    const float rc_hs = 1.0f / sp.fhs, rc_ws = 1.0f / sp.fws;
    PadGeom pg;
    pg.Wp = Ws + 2 * kPad;
    pg.row = pg.Wp * 16;
    pg.org = (kPad * pg.Wp + kPad) * 16;
    pg.plane_bytes = (int)((int64_t)(Hs + 2 * kPad) * pg.Wp * 16);
    const float4* im = reinterpret_cast<const float4*>(img4);
    const dim3 grid(blocks(per_view, 256), B, 1);
    // 16-B group stores need 16-B aligned output rows; the LDS-staged store needs the
    // dense volume layout (each view one contiguous run of items)
    const bool vec = aligned16(out) && out_pstride % 4 == 0 && out_bstride % 4 == 0;
    const bool dense = vec && out_pstride == (int64_t)NG * kSweepDG * C;
    int store = dense ? 2 : vec ? 1 : 0;
    const int o_store = opt(kOptSweepStore);  // A/B only: the grouped kernel's store modes
    const bool grouped = o_store >= 0;
    // the depth-per-lane kernel reads the depths from global memory (any D); the pixel-per-lane
    // one stages them in LDS (D <= kSweepMaxLdsD, else the tile kernel)
    const bool tile = !grouped && (opt(kOptSweepTile) || (D > kSweepMaxLdsD && opt(kOptSweepDlane) == 0));
    if (grouped) store = min(store, o_store);
    hipStream_t q = S(stream);
    if (!grouped && !tile) {
        // default: source footprint staged in LDS (plane_sweep_lds_kernel)
        const int64_t tiles = (int64_t)((Wt + kSLP - 1) / kSLP) * ((Ht + kSLR - 1) / kSLR);
        if (tiles > kMaxGridX) return fail(MPIV_ERR_ARG, "mpiv_plane_sweep_padded: too large");
        const dim3 lgrid((unsigned)tiles, B, 1);
        const int shrink = opt(kOptBoxShrink);
        [[maybe_unused]] const FastDiv fd_b = make_fastdiv((unsigned)(16 * NG));
        if (opt(kOptSweepDlane) != 0) {
#define MPIV_DLANE(CC)                                                                                          \
    plane_sweep_dlane_kernel<CC, false><<<lgrid, kDLThreads, 0, q>>>(im, pg, nullptr, ImgStrides{0, 0, 0, 0}, sp, \
                                                                     rc_hs, rc_ws, ki, proj, depths, out,          \
                                                                     out_bstride, out_pstride, (int)vec, shrink)
            switch (C) {
                case 1: MPIV_DLANE(1); break;
                case 2: MPIV_DLANE(2); break;
                case 3: MPIV_DLANE(3); break;
                default: MPIV_DLANE(4); break;
            }
#undef MPIV_DLANE
            return launched("mpiv_plane_sweep_padded");
        }
#if MPIV_AB  // pixel-per-lane LDS, tile and grouped sweeps (A/B)
#define MPIV_LDS(CC)                                                                                          \
    plane_sweep_lds_kernel<CC><<<lgrid, kSLThreads, 0, q>>>(im, sp, pg, rc_hs, rc_ws, fd_g, fd_b, ki, proj, depths, \
                                                     out, out_bstride, out_pstride, (int)vec, shrink)
        switch (C) {
            case 1: MPIV_LDS(1); break;
            case 2: MPIV_LDS(2); break;
            case 3: MPIV_LDS(3); break;
            default: MPIV_LDS(4); break;
        }
#undef MPIV_LDS
        return launched("mpiv_plane_sweep_padded");
    }
    if (tile) {
        const int npix = Ht * Wt;
        const int last = D - ((D - 1) / kTileD) * kTileD;  // depths in the last chunk
        const dim3 tgrid(blocks(npix, kTileP), B, 1);
        const FastDiv fw = make_fastdiv((unsigned)Wt), ff = make_fastdiv((unsigned)(kTileD * C)),
                      fl = make_fastdiv((unsigned)(last * C));
#define MPIV_TILE(CC)                                                                                            \
    plane_sweep_tile_kernel<CC><<<tgrid, 256, 0, q>>>(im, sp, pg, rc_hs, rc_ws, fw, ff, fl, ki, proj, depths, out, \
                                                      out_bstride, out_pstride)
        switch (C) {
            case 1: MPIV_TILE(1); break;
            case 2: MPIV_TILE(2); break;
            case 3: MPIV_TILE(3); break;
            default: MPIV_TILE(4); break;
        }
#undef MPIV_TILE
        return launched("mpiv_plane_sweep_padded");
    }
#define MPIV_SWEEP(CC, VV)                                                                                  \
    plane_sweep_group_kernel<CC, VV><<<grid, 256, 0, q>>>(im, sp, pg, rc_hs, rc_ws, fd_g, fd_w, ki, proj, depths, \
                                                          out, out_bstride, (int)out_pstride)
#define MPIV_SWEEP_C(CC)                   \
    if (store == 2) MPIV_SWEEP(CC, 2);     \
    else if (store == 1) MPIV_SWEEP(CC, 1); \
    else MPIV_SWEEP(CC, 0)
    switch (C) {
        case 1: MPIV_SWEEP_C(1); break;
        case 2: MPIV_SWEEP_C(2); break;
        case 3: MPIV_SWEEP_C(3); break;
        default: MPIV_SWEEP_C(4); break;
    }
#undef MPIV_SWEEP_C
#undef MPIV_SWEEP
    return launched("mpiv_plane_sweep_padded");
#else
    }
    return fail(MPIV_ERR_ARG, "mpiv_plane_sweep_padded: an A/B sweep kernel, built only into libmpiv_ab.so");
#endif
}

int mpiv_plane_sweep_padded(const float* img4, int B, int Hs, int Ws, int C, const float* ki, const float* proj,
                            const float* depths, int D, int Ht, int Wt, float* out, void* stream) {
    return mpiv_plane_sweep_padded_into(img4, B, Hs, Ws, C, ki, proj, depths, D, Ht, Wt, out,
                                        (int64_t)Ht * Wt * D * C, (int64_t)D * C, stream);
}

int mpiv_inverse_warp(const float* img, const int64_t st[4], int B, int Hs, int Ws, int C, const float* ki,
                      const float* proj, const float* depth, const int64_t dst[3], int Ht, int Wt, float* out,
                      void* stream) {
    if (!img || !st || !ki || !proj || !depth || !dst || !out)
        return fail(MPIV_ERR_ARG, "mpiv_inverse_warp: null pointer");
    if (B <= 0 || Hs <= 0 || Ws <= 0 || C <= 0 || Ht <= 0 || Wt <= 0)
        return fail(MPIV_ERR_ARG, "mpiv_inverse_warp: bad shape");
    if (B > kMaxGridYZ) return fail(MPIV_ERR_ARG, "mpiv_inverse_warp: too large");
    const ImgStrides s{st[0], st[1], st[2], st[3]};
    dim3 grid(blocks((int64_t)Ht * Wt, 256), B, 1);
    inverse_warp_kernel<<<grid, 256, 0, S(stream)>>>(img, s, sweep_params(B, Hs, Ws, C, 1, Ht, Wt), ki, proj, depth,
                                                     dst[0], dst[1], dst[2], out);
    return launched("mpiv_inverse_warp");
}

int mpiv_grid_sample(const float* in, const int64_t ist[4], int N, int C, int Hi, int Wi, const float* coords,
                     const int64_t cst[4], int Ho, int Wo, float* out, const int64_t ost[4], void* stream) {
    if (!in || !ist || !coords || !cst || !out || !ost) return fail(MPIV_ERR_ARG, "mpiv_grid_sample: null pointer");
    if (N <= 0 || C <= 0 || Hi <= 0 || Wi <= 0 || Ho <= 0 || Wo <= 0)
        return fail(MPIV_ERR_ARG, "mpiv_grid_sample: bad shape");
    if (N > kMaxGridYZ) return fail(MPIV_ERR_ARG, "mpiv_grid_sample: too large");
    const Strides4 is{ist[0], ist[1], ist[2], ist[3]};
    // coords strides arrive as (n, y, x, component); the kernel reads them as
    // {n, c=component, y, x}
    const Strides4 cs{cst[0], cst[3], cst[1], cst[2]};
    const Strides4 os{ost[0], ost[1], ost[2], ost[3]};
    dim3 grid(blocks((int64_t)Ho * Wo, 256), N, 1);
    grid_sample_kernel<<<grid, 256, 0, S(stream)>>>(in, is, C, Hi, Wi, coords, cs, Ho, Wo, out, os);
    return launched("mpiv_grid_sample");
}

int mpiv_over_composite(const float* const* layers, int P, int64_t n, int64_t ps, int64_t cs, float* out,
                        void* stream) {
    if (!layers || !out) return fail(MPIV_ERR_ARG, "mpiv_over_composite: null pointer");
    if (P <= 0 || n <= 0) return fail(MPIV_ERR_ARG, "mpiv_over_composite: bad shape");
    over_composite_kernel<<<blocks(n, 256), 256, 0, S(stream)>>>(layers, P, n, ps, cs, out);
    return launched("mpiv_over_composite");
}

int mpiv_transform_points(const float* pts, int M, int64_t n, const float* homs, float* out, void* stream) {
    if (!pts || !homs || !out) return fail(MPIV_ERR_ARG, "mpiv_transform_points: null pointer");
    if (M <= 0 || n <= 0 || M > kMaxGridYZ) return fail(MPIV_ERR_ARG, "mpiv_transform_points: bad shape");
    transform_points_kernel<<<dim3(blocks(n, 256), M), 256, 0, S(stream)>>>(pts, n, homs, out);
    return launched("mpiv_transform_points");
}

int mpiv_normalize_homogeneous(float* pts, int64_t n, int k, float* out, void* stream) {
    if (!pts || !out) return fail(MPIV_ERR_ARG, "mpiv_normalize_homogeneous: null pointer");
    if (n <= 0 || k <= 0) return fail(MPIV_ERR_ARG, "mpiv_normalize_homogeneous: bad shape");
    normalize_homogeneous_kernel<<<blocks(n, 256), 256, 0, S(stream)>>>(pts, n, k, out);
    return launched("mpiv_normalize_homogeneous");
}

int mpiv_pixel2cam(const float* depth, const float* pix, const float* ki, int B, int64_t n, int homogeneous,
                   float* cam, void* stream) {
    if (!depth || !pix || !ki || !cam) return fail(MPIV_ERR_ARG, "mpiv_pixel2cam: null pointer");
    if (B <= 0 || n <= 0 || B > kMaxGridYZ) return fail(MPIV_ERR_ARG, "mpiv_pixel2cam: bad shape");
    pixel2cam_kernel<<<dim3(blocks(n, 256), B), 256, 0, S(stream)>>>(depth, pix, ki, n, homogeneous, cam);
    return launched("mpiv_pixel2cam");
}

int mpiv_cam2pixel(const float* cam, const float* proj, int B, int64_t n, float* out, void* stream) {
    if (!cam || !proj || !out) return fail(MPIV_ERR_ARG, "mpiv_cam2pixel: null pointer");
    if (B <= 0 || n <= 0 || B > kMaxGridYZ) return fail(MPIV_ERR_ARG, "mpiv_cam2pixel: bad shape");
    cam2pixel_kernel<<<dim3(blocks(n, 256), B), 256, 0, S(stream)>>>(cam, proj, n, out);
    return launched("mpiv_cam2pixel");
}

int mpiv_plane_coords(const float* pts, int M, int64_t n, const float* homs, int Ht, int Wt, float* coords,
                      void* stream) {
    if (!pts || !homs || !coords) return fail(MPIV_ERR_ARG, "mpiv_plane_coords: null pointer");
    if (M <= 0 || n <= 0 || M > kMaxGridYZ || Ht <= 0 || Wt <= 0)
        return fail(MPIV_ERR_ARG, "mpiv_plane_coords: bad shape");
    plane_coords_kernel<<<dim3(blocks(n, 256), M), 256, 0, S(stream)>>>(pts, n, homs, (float)(Ht - 1),
                                                                        (float)(Wt - 1), coords);
    return launched("mpiv_plane_coords");
}

int mpiv_preprocess(const float* in, int64_t n, float* out, void* stream) {
    if (!in || !out) return fail(MPIV_ERR_ARG, "mpiv_preprocess: null pointer");
    if (n <= 0) return fail(MPIV_ERR_ARG, "mpiv_preprocess: bad size");
    preprocess_kernel<<<blocks(n, 256), 256, 0, S(stream)>>>(in, n, out);
    return launched("mpiv_preprocess");
}

int mpiv_deprocess_u8(const float* in, int64_t n, uint8_t* out, void* stream) {
    if (!in || !out) return fail(MPIV_ERR_ARG, "mpiv_deprocess_u8: null pointer");
    if (n <= 0) return fail(MPIV_ERR_ARG, "mpiv_deprocess_u8: bad size");
    deprocess_u8_kernel<<<blocks(n, 256), 256, 0, S(stream)>>>(in, n, out);
    return launched("mpiv_deprocess_u8");
}

// ---- MPI assembly from the network output (ipynb cell 10 L79-111) ----------------

static int check_net(const char* nm, const float* pred, const int64_t ps[4], const float* fg, const int64_t fs[4],
                     int B, int H, int W, int P) {
    if (!pred || !ps || !fg || !fs) return fail(MPIV_ERR_ARG, "%s: null pointer", nm);
    if (B <= 0 || H <= 0 || W <= 0 || P <= 0) return fail(MPIV_ERR_ARG, "%s: bad shape", nm);
    if ((int64_t)H * W >= (1ll << 31) || B > kMaxGridYZ) return fail(MPIV_ERR_ARG, "%s: too large", nm);
    return MPIV_OK;
}

int mpiv_assemble_mpi(const float* pred, const int64_t ps[4], const float* fg, const int64_t fs[4], int B, int H,
                      int W, int P, float* rgba, void* stream) {
    if (int rc = check_net("mpiv_assemble_mpi", pred, ps, fg, fs, B, H, W, P)) return rc;
    if (!rgba || !aligned16(rgba)) return fail(MPIV_ERR_ARG, "mpiv_assemble_mpi: rgba null or not 16-byte aligned");
    if (blocks(P, kAsmPl) > kMaxGridYZ) return fail(MPIV_ERR_ARG, "mpiv_assemble_mpi: too many planes");
    const NetStrides s{ps[0], ps[1], ps[2], ps[3], fs[0], fs[1], fs[2], fs[3]};
    const dim3 grid(blocks((int64_t)H * W, kAsmPix), blocks(P, kAsmPl), B);
    assemble_native_kernel<<<grid, 256, 0, S(stream)>>>(pred, fg, s, H, W, P, make_fastdiv((unsigned)W),
                                                        reinterpret_cast<float4*>(rgba));
    return launched("mpiv_assemble_mpi");
}

// mpiv_assemble_mpi for a render's backward only (round 6, the fused net-output training's
// re-assembly): the texel rows no output pixel of the render of `homs` ([B][P][9], the render's
// own) can sample are left unwritten -- the chain reads in-image taps only, inside those rows.
int mpiv_assemble_mpi_sampled(const float* pred, const int64_t ps[4], const float* fg, const int64_t fs[4], int B,
                              int H, int W, int P, const float* homs, float* rgba, void* stream) {
    if (int rc = check_net("mpiv_assemble_mpi_sampled", pred, ps, fg, fs, B, H, W, P)) return rc;
    if (!rgba || !aligned16(rgba) || !homs)
        return fail(MPIV_ERR_ARG, "mpiv_assemble_mpi_sampled: rgba / homs null or rgba not 16-byte aligned");
    if (blocks(P, kAsmPl) > kMaxGridYZ) return fail(MPIV_ERR_ARG, "mpiv_assemble_mpi_sampled: too many planes");
    const NetStrides s{ps[0], ps[1], ps[2], ps[3], fs[0], fs[1], fs[2], fs[3]};
    const dim3 grid(blocks((int64_t)H * W, kAsmPix), blocks(P, kAsmPl), B);
    // the bounds use the render's fast position recipe (H, W >= 2); smaller frames assemble every row
    const bool rows = H >= 2 && W >= 2;
    assemble_native_kernel<<<grid, 256, 0, S(stream)>>>(pred, fg, s, H, W, P, make_fastdiv((unsigned)W),
                                                        reinterpret_cast<float4*>(rgba), rows ? homs : nullptr,
                                                        rows ? make_geom(H, W, P) : RenderGeom{});
    return launched("mpiv_assemble_mpi_sampled");
}

int mpiv_assemble_mpi_packed(const float* pred, const int64_t ps[4], const float* fg, const int64_t fs[4], int b,
                             int H, int W, int P, float* packed, void* stream) {
    if (int rc = check_net("mpiv_assemble_mpi_packed", pred, ps, fg, fs, b + 1, H, W, P)) return rc;
    if (b < 0) return fail(MPIV_ERR_ARG, "mpiv_assemble_mpi_packed: bad batch index");
    if (!packed || !aligned16(packed))
        return fail(MPIV_ERR_ARG, "mpiv_assemble_mpi_packed: packed null or not 16-byte aligned");
    if ((int64_t)(H + 2 * kPad) * (W + 2 * kPad) * 16 >= (int64_t)kOOB || P > kMaxGridYZ)
        return fail(MPIV_ERR_ARG, "mpiv_assemble_mpi_packed: padded plane larger than 2 GiB or too many planes");
    const NetStrides s{ps[0], ps[1], ps[2], ps[3], fs[0], fs[1], fs[2], fs[3]};
    const int64_t npix = (int64_t)(H + 2 * kPad) * (W + 2 * kPad);
    assemble_packed_kernel<<<dim3(blocks(npix, 256), P), 256, 0, S(stream)>>>(
        pred, fg, s, H, W, P, b, make_fastdiv((unsigned)(W + 2 * kPad)), reinterpret_cast<float4*>(packed), npix);
    return launched("mpiv_assemble_mpi_packed");
}

int mpiv_assemble_mpi_backward(const float* drgba, const int64_t gs[5], const float* pred, const int64_t ps[4],
                               const float* fg, const int64_t fs[4], int B, int H, int W, int P, float* dpred,
                               float* dfg, void* stream) {
    if (int rc = check_net("mpiv_assemble_mpi_backward", pred, ps, fg, fs, B, H, W, P)) return rc;
    if (!drgba || !gs || !dpred) return fail(MPIV_ERR_ARG, "mpiv_assemble_mpi_backward: null pointer");
    const NetStrides s{ps[0], ps[1], ps[2], ps[3], fs[0], fs[1], fs[2], fs[3]};
    const NativeStrides g{gs[0], gs[1], gs[2], gs[3], gs[4]};
    const bool dense = g.c == 1 && g.p == 4 && g.x == (int64_t)P * 4 && g.y == (int64_t)W * P * 4 &&
                       g.b == (int64_t)H * W * P * 4 && aligned16(drgba);
    if (dense)
        assemble_backward_dense_kernel<<<dim3(blocks((int64_t)H * W, kAbPix), B), kAbPix, 0, S(stream)>>>(
            reinterpret_cast<const float4*>(drgba), pred, fg, s, H, W, P, make_fastdiv((unsigned)W), dpred, dfg);
    else
        assemble_backward_kernel<<<dim3(blocks((int64_t)H * W, 256), B), 256, 0, S(stream)>>>(
            drgba, g, pred, fg, s, H, W, P, make_fastdiv((unsigned)W), dpred, dfg);
    return launched("mpiv_assemble_mpi_backward");
}

// render_netout_kernel's geometry (netout_geo = 100 * waves + 10 * rows + depth; automatic: 821)
// netout_geo: waves * 100 + rows * 10 + planes of w / a in flight; + 1000: the double-buffered box (DB)
static int netout_geo() {
    const int o = opt(kOptNetoutGeo);
    switch (o) {
        case 811: case 821: case 822: case 422: case 1821: return o;
        default: return 1821;  // round 5: double-buffered box, one barrier per plane (0.110-0.116 vs 0.115-0.122 ms)
    }
}

// The assembly fused into the render (assemble.hip render_netout_kernel): pred/fg -> frames
// (and, ckpt != nullptr, the training forward's composite checkpoints).
static int render_net_output_impl(const char* nm, const float* pred, const int64_t ps[4], const float* fg,
                                  const int64_t fs[4], int B, int H, int W, int P, const float* homs, float* out,
                                  float* ckpt_f, void* stream) {
    float4* ckpt = reinterpret_cast<float4*>(ckpt_f);
    if (int rc = check_net(nm, pred, ps, fg, fs, B, H, W, P)) return rc;
    if (!homs || !out) return fail(MPIV_ERR_ARG, "%s: null pointer", nm);
    if (ckpt && !aligned16(ckpt)) return fail(MPIV_ERR_ARG, "%s: ckpt not 16-byte aligned", nm);
    if (H < 2 || W < 2 || H >= (1 << 15) - 4 || W >= (1 << 15) - 4 || P > kNMaxP)
        return fail(MPIV_ERR_ARG, "%s: needs 2 <= H, W < 32764 and P <= %d", nm, kNMaxP);
    const NetStrides s{ps[0], ps[1], ps[2], ps[3], fs[0], fs[1], fs[2], fs[3]};
    const RenderGeom g = make_geom(H, W, P);
    const int geo = netout_geo();
    const int NW = geo / 100 % 10, R = geo / 10 % 10;
    const bool db = geo >= 1000;
    const int64_t nb = (int64_t)blocks(W, kNTX) * blocks(H, NW * R) * B;
    if (nb > kMaxGridX) return fail(MPIV_ERR_ARG, "%s: too many blocks", nm);
    // buffer addressing when one batch element's pred / fg spans fit a 32-bit byte offset
    NetStrides sb = s;
    const int64_t pspan = ((int64_t)(2 * P + 2) * ps[1] + (int64_t)(H - 1) * ps[2] + (int64_t)(W - 1) * ps[3] + 1) * 4;
    const int64_t fspan = ((int64_t)(H - 1) * fs[1] + (int64_t)(W - 1) * fs[2] + 2 * fs[3] + 1) * 4;
    const bool buf = opt(kOptNetoutBuf) != 0 && pspan < (int64_t)kOOB && fspan < (int64_t)kOOB;
    if (buf) {
        sb.pred_bytes = (int)pspan;
        sb.fg_bytes = (int)fspan;
    }
    // the reference image's channels contiguous: one 12-B colour load per staged texel (netout_fg3=0: three)
    const bool fg3 = buf && db && fs[3] == 1 && opt(kOptNetoutFg3) != 0;
    if (g_route) {
        if (fg3)
            return note_route(nb, 64 * NW, "render_netout_kernel<%d, %d, %d, true, true, true>", NW, R, geo % 10);
        return note_route(nb, 64 * NW, "render_netout_kernel<%d, %d, %d, %s, %s>", NW, R, geo % 10, buf ? "true" : "false",
                          db ? "true" : "false");
    }
    const unsigned nbu = (unsigned)nb;
    hipStream_t q = S(stream);
    switch (geo * 2 + (buf ? 1 : 0)) {
#define MPIV_NETOUT(A, B_, C, D)                                                                           \
    case (A * 100 + B_ * 10 + C) * 2 + D:                                                                  \
        render_netout_kernel<A, B_, C, D><<<nbu, 64 * A, 0, q>>>(pred, fg, sb, g, B, homs, out, ckpt);     \
        break;
        MPIV_NETOUT(8, 1, 1, 0) MPIV_NETOUT(8, 2, 1, 0) MPIV_NETOUT(8, 2, 2, 0) MPIV_NETOUT(4, 2, 2, 0)
        MPIV_NETOUT(8, 1, 1, 1) MPIV_NETOUT(8, 2, 1, 1) MPIV_NETOUT(8, 2, 2, 1) MPIV_NETOUT(4, 2, 2, 1)
#undef MPIV_NETOUT
        case 1821 * 2:
            render_netout_kernel<8, 2, 1, false, true><<<nbu, 512, P * sizeof(int2), q>>>(pred, fg, sb, g, B, homs, out,
                                                                                           ckpt);
            break;
        case 1821 * 2 + 1:
            if (fg3)
                render_netout_kernel<8, 2, 1, true, true, true><<<nbu, 512, P * sizeof(int2), q>>>(pred, fg, sb, g, B, homs,
                                                                                                out, ckpt);
            else
                render_netout_kernel<8, 2, 1, true, true><<<nbu, 512, P * sizeof(int2), q>>>(pred, fg, sb, g, B, homs, out,
                                                                                              ckpt);
            break;
    }
    return launched(nm);
}

int mpiv_render_net_output(const float* pred, const int64_t ps[4], const float* fg, const int64_t fs[4], int B, int H,
                           int W, int P, const float* homs, float* out, void* stream) {
    return render_net_output_impl("mpiv_render_net_output", pred, ps, fg, fs, B, H, W, P, homs, out, nullptr, stream);
}

int mpiv_render_net_output_train(const float* pred, const int64_t ps[4], const float* fg, const int64_t fs[4], int B,
                                 int H, int W, int P, const float* homs, float* out, float* ckpt, void* stream) {
    if (!ckpt) return fail(MPIV_ERR_ARG, "mpiv_render_net_output_train: null ckpt");
    return render_net_output_impl("mpiv_render_net_output_train", pred, ps, fg, fs, B, H, W, P, homs, out, ckpt,
                                  stream);
}

// ---- host-side homographies (inv_homography_torch chain, utils.py:44-67) -------------
// The reference evaluates the chain with torch-CPU ops on materialised [P,B,...] tensors;
// torch's CPU matmul of these tiny matrices rounds as plain products summed in ascending
// k (no FMA; checked against torch for every shape of the chain, batch 1..1280), and the
// rest is elementwise IEEE arithmetic, so the chain is restated here exactly (the library
// builds with -ffp-contract=off, host code included).  Kinv = torch.inverse(K) comes from
// the caller (LAPACK).  Pinned bit-exact by tests/test_host.py against the reference's H.
int mpiv_render_homographies(const float* pose, const float* depths, const float* K, const float* Kinv, int B,
                             int P, float* H) {
    if (!pose || !depths || !K || !Kinv || !H) return fail(MPIV_ERR_ARG, "mpiv_render_homographies: null pointer");
    if (B <= 0 || P <= 0) return fail(MPIV_ERR_ARG, "mpiv_render_homographies: bad shape");
    for (int b = 0; b < B; ++b)
        for (int p = 0; p < P; ++p) render_hom_chain(pose + (int64_t)b * 16, depths[p], K + (int64_t)b * 9,
                                                     Kinv + (int64_t)b * 9, H + ((int64_t)b * P + p) * 9);
    g_err[0] = '\0';
    return MPIV_OK;
}

// The same chain on the device, one work-item per (view, plane), for poses / intrinsics
// that already live in HBM (no blocking device-to-host copies on the render path).
// Same code as the host entry (render_hom_chain, IEEE fp32, no contraction, correctly
// rounded division): bit-identical results (tests/test_host.py).
int mpiv_render_homographies_device(const float* pose, const float* depths, const float* K, const float* Kinv,
                                    int B, int P, float* H, void* stream) {
    const char* nm = "mpiv_render_homographies_device";
    if (!pose || !depths || !K || !Kinv || !H) return fail(MPIV_ERR_ARG, "%s: null pointer", nm);
    if (B <= 0 || P <= 0 || (int64_t)B * P >= (1ll << 31)) return fail(MPIV_ERR_ARG, "%s: bad shape", nm);
    render_homographies_kernel<<<blocks((int64_t)B * P, 256), 256, 0, S(stream)>>>(pose, depths, K, Kinv, B, P, H);
    return launched(nm);
}

// proj = [[K_src, 0], [0, 0, 0, 1]] @ pose for projective_inverse_warp_torch[2] (utils.py:428-438,
// 747-757), torch-CPU rounding restated (geometry.hip psv_proj): on the host ...
int mpiv_psv_proj(const float* Ks, int64_t ks_bstride, const float* pose, int B, float* proj) {
    if (!Ks || !pose || !proj) return fail(MPIV_ERR_ARG, "mpiv_psv_proj: null pointer");
    if (B <= 0 || ks_bstride < 0) return fail(MPIV_ERR_ARG, "mpiv_psv_proj: bad shape");
    for (int b = 0; b < B; ++b) psv_proj(Ks + (int64_t)b * ks_bstride, pose + (int64_t)b * 16, proj + (int64_t)b * 16);
    g_err[0] = '\0';
    return MPIV_OK;
}

// ... and on the device, for poses / intrinsics already in HBM (the notebook's dataset call,
// ipynb cell 8 L49-75): no device-to-host copy; bit-identical to the host entry
int mpiv_psv_proj_device(const float* Ks, int64_t ks_bstride, const float* pose, int B, float* proj, void* stream) {
    const char* nm = "mpiv_psv_proj_device";
    if (!Ks || !pose || !proj) return fail(MPIV_ERR_ARG, "%s: null pointer", nm);
    if (B <= 0 || ks_bstride < 0) return fail(MPIV_ERR_ARG, "%s: bad shape", nm);
    psv_proj_kernel<<<blocks(B, 64), 64, 0, S(stream)>>>(Ks, ks_bstride, pose, B, proj);
    return launched(nm);
}

int mpiv_synth_mpi_packed(uint32_t seed, int H, int W, int p_begin, int p_end, float* packed, void* stream) {
    const char* nm = "mpiv_synth_mpi_packed";
    if (!packed) return fail(MPIV_ERR_ARG, "%s: null pointer", nm);
    if (H <= 0 || W <= 0 || p_begin < 0 || p_end <= p_begin) return fail(MPIV_ERR_ARG, "%s: bad shape", nm);
    if (!aligned16(packed)) return fail(MPIV_ERR_ARG, "%s: packed must be 16-byte aligned", nm);
    if ((int64_t)(H + 2 * kPad) * (W + 2 * kPad) * 16 >= (int64_t)kOOB || (int64_t)H * W >= (1ll << 31) ||
        p_end - p_begin > kMaxGridYZ)
        return fail(MPIV_ERR_ARG, "%s: padded plane larger than 2 GiB or too many planes", nm);
    const int64_t npix = (int64_t)(H + 2 * kPad) * (W + 2 * kPad);
    synth_packed_kernel<<<dim3(blocks(npix, 256), p_end - p_begin), 256, 0, S(stream)>>>(
        seed, H, W, p_begin, make_fastdiv((unsigned)(W + 2 * kPad)), reinterpret_cast<float4*>(packed), npix);
    return launched(nm);
}

// ---- 8-bit RGBA MPI (render_u8.hip) -------------------------------------------------

int mpiv_pack_planes_u8(const uint8_t* mpi, const int64_t st[4], int H, int W, int P, uint32_t* packed,
                        void* stream) {
    const char* nm = "mpiv_pack_planes_u8";
    if (!mpi || !st || !packed) return fail(MPIV_ERR_ARG, "%s: null pointer", nm);
    if (H <= 0 || W <= 0 || P <= 0) return fail(MPIV_ERR_ARG, "%s: bad shape", nm);
    if (reinterpret_cast<uintptr_t>(packed) & 3) return fail(MPIV_ERR_ARG, "%s: packed must be 4-byte aligned", nm);
    const int64_t npix = (int64_t)(H + 2 * kPad) * (W + 2 * kPad);
    if (npix * 4 >= (int64_t)kOOB || blocks(P, kPackPl) > kMaxGridYZ)
        return fail(MPIV_ERR_ARG, "%s: padded plane larger than 2 GiB or too many planes", nm);
    const NativeStrides s{0, st[0], st[1], st[2], st[3]};
    pack_planes_u8_kernel<<<dim3(blocks(npix, kPackPix), blocks(P, kPackPl)), 256, 0, S(stream)>>>(
        mpi, s, H, W, P, make_fastdiv((unsigned)(W + 2 * kPad)), packed, npix);
    return launched(nm);
}

int mpiv_unpack_planes_u8(const uint32_t* packed, int H, int W, int P, float* out, void* stream) {
    const char* nm = "mpiv_unpack_planes_u8";
    if (!packed || !out) return fail(MPIV_ERR_ARG, "%s: null pointer", nm);
    if (H <= 0 || W <= 0 || P <= 0) return fail(MPIV_ERR_ARG, "%s: bad shape", nm);
    if ((reinterpret_cast<uintptr_t>(packed) & 3) || !aligned16(out))
        return fail(MPIV_ERR_ARG, "%s: alignment (packed 4 B, out 16 B)", nm);
    const int64_t n = (int64_t)P * (H + 2 * kPad) * (W + 2 * kPad);
    const int64_t nb = std::min<int64_t>(blocks(n, 256), 1 << 20);
    unpack_u8_planes_kernel<<<(unsigned)nb, 256, 0, S(stream)>>>(packed, reinterpret_cast<float4*>(out), n);
    return launched(nm);
}

int mpiv_synth_mpi_packed_u8(uint32_t seed, int H, int W, int p_begin, int p_end, uint32_t* packed, void* stream) {
    const char* nm = "mpiv_synth_mpi_packed_u8";
    if (!packed) return fail(MPIV_ERR_ARG, "%s: null pointer", nm);
    if (H <= 0 || W <= 0 || p_begin < 0 || p_end <= p_begin) return fail(MPIV_ERR_ARG, "%s: bad shape", nm);
    if (reinterpret_cast<uintptr_t>(packed) & 3) return fail(MPIV_ERR_ARG, "%s: packed must be 4-byte aligned", nm);
    const int64_t npix = (int64_t)(H + 2 * kPad) * (W + 2 * kPad);
    if (npix * 4 >= (int64_t)kOOB || (int64_t)H * W >= (1ll << 31) || p_end - p_begin > kMaxGridYZ)
        return fail(MPIV_ERR_ARG, "%s: padded plane larger than 2 GiB or too many planes", nm);
    synth_packed_u8_kernel<<<dim3(blocks(npix, 256), p_end - p_begin), 256, 0, S(stream)>>>(
        seed, H, W, p_begin, make_fastdiv((unsigned)(W + 2 * kPad)), packed, npix);
    return launched(nm);
}

static int render_u8_impl(const uint32_t* packed, int H, int W, int P, int p_begin, int p_end, int back,
                          const float* homs, int V, float* out, bool ct, void* stream) {
    const char* nm = ct ? "mpiv_render_packed_u8_ct" : "mpiv_render_packed_u8";
    if (!packed || !homs || !out) return fail(MPIV_ERR_ARG, "%s: null pointer", nm);
    if (V <= 0 || H < 2 || W < 2 || P <= 0) return fail(MPIV_ERR_ARG, "%s: bad shape (H, W >= 2)", nm);
    if (p_begin < 0 || p_end > P || p_begin >= p_end) return fail(MPIV_ERR_ARG, "%s: bad plane range", nm);
    if ((reinterpret_cast<uintptr_t>(packed) & 3) || (ct && !aligned16(out)))
        return fail(MPIV_ERR_ARG, "%s: alignment (packed 4 B, ct 16 B)", nm);
    const int64_t npix = (int64_t)(H + 2 * kPad) * (W + 2 * kPad);
    if (npix * 4 >= (int64_t)kOOB || H >= (1 << 22) || W >= (1 << 22))
        return fail(MPIV_ERR_ARG, "%s: padded plane larger than 2 GiB or a side >= 2^22", nm);
    const RenderGeom g = make_geom(H, W, P);
    U8Geom ug;
    ug.row = g.Wp * 4;
    ug.org = (kPad * g.Wp + kPad) * 4;
    ug.plane_bytes = (int)(npix * 4);
    // automatic: 4 rows per work-item with vertical tap reuse (the north taps' u8 -> float
    // conversions are reused too): 8 views 1.93 vs 2.17 ms, 125 views 30.0 vs 33.2 ms, single
    // view 0.337 vs 0.340, config-5 shard 0.611 vs 0.620 for 2 plain rows (profiles/r02_u8_render.jsonl).
    // A/B: render_tile=2|8 plain rows; render_tile=4|8 with render_vshare=1: reuse, that many rows
    // Stretched MPIs (swapped x/(H-1) normalisation) take it only when the launch fills the chip
    // (>= 2048 tiles of 64x32, as the float route): config 2 at one view 0.080-0.089 vs 0.065 ms
    // for 2 plain rows, at 64 views 2.35 vs 2.40-2.49.
    const float sxr = (float)W / (float)(H - 1), syr = (float)H / (float)(W - 1);
    const bool square = sxr >= 0.8f && sxr <= 1.25f && syr >= 0.8f && syr <= 1.25f;
    const bool big = (int64_t)blocks(W, kTileX) * blocks(H, 4 * 8) * V >= 2048;
    const int rt = opt(kOptRenderTile), vso = opt(kOptRenderVshare);
    // render_tile: 0 automatic, -1 / 2 two plain rows, 8 eight plain rows, 4 | 8 with render_vshare=1
    if (!(rt == 0 || rt == -1 || rt == 2 || rt == 8 || (rt == 4 && vso == 1)))
        return fail(MPIV_ERR_ARG, "%s: render_tile=%d (render_vshare=%d) is not a u8 render variant", nm, rt, vso);
    const bool vs = (rt == 0 && vso != -1 && (square || big)) || (vso == 1 && (rt == 4 || rt == 8));
    const int R = rt == 0 ? (vs ? 4 : 2) : vs ? rt : rt == 8 ? 8 : 2;
    const int64_t nb = (int64_t)blocks(W, kTileX) * blocks(H, 4 * R) * V;
    if (nb > kMaxGridX) return fail(MPIV_ERR_ARG, "%s: too many blocks", nm);
    if (g_route) {  // every template argument, as rocprof's demangled name shows it
        const int f = opt(kOptU8Flight) ? opt(kOptU8Flight) : (nb < 2048 ? 4 : 2);
        const int d = (vs && R == 4 && (f == 4 || f == 8)) ? f : 2;
        return note_route(nb, 256, "render_u8_kernel<%s, %d, %s, %d>", ct ? "true" : "false", R, vs ? "true" : "false", d);
    }
    const unsigned* pk = reinterpret_cast<const unsigned*>(packed);
    hipStream_t q = S(stream);
#define MPIV_U8(CT, RR, VV)                                                                                       \
    render_u8_kernel<CT, RR, VV><<<(unsigned)nb, 256, 0, q>>>(pk, npix, g, ug, V, p_begin, p_end, CT ? back : 1, \
                                                              homs, out)
#if MPIV_AB  // 8 rows per work-item (A/B)
    if (R == 8) {
        if (vs && ct) MPIV_U8(true, 8, true);
        else if (vs) MPIV_U8(false, 8, true);
        else if (ct) MPIV_U8(true, 8, false);
        else MPIV_U8(false, 8, false);
        return launched(nm);
    }
#endif
    // 4 rows in flight when the launch leaves the SIMDs few waves (one view: 1024 blocks = 4 waves
    // per SIMD; 0.32 vs 0.37 ms), 2 for large launches (125 views: 30.2 vs 30.5 ms; r04j_strips_ab.jsonl)
    const int u8f = opt(kOptU8Flight) ? opt(kOptU8Flight) : (nb < 2048 ? 4 : 2);
    if (vs && u8f == 8) {  // 8 rows in flight (two planes' rows)
        if (ct) render_u8_kernel<true, 4, true, 8><<<(unsigned)nb, 256, 0, q>>>(pk, npix, g, ug, V, p_begin, p_end, back,
                                                                              homs, out);
        else render_u8_kernel<false, 4, true, 8><<<(unsigned)nb, 256, 0, q>>>(pk, npix, g, ug, V, p_begin, p_end, 1,
                                                                             homs, out);
    } else if (vs && u8f == 4) {  // 4 rows in flight
        if (ct) render_u8_kernel<true, 4, true, 4><<<(unsigned)nb, 256, 0, q>>>(pk, npix, g, ug, V, p_begin, p_end, back,
                                                                              homs, out);
        else render_u8_kernel<false, 4, true, 4><<<(unsigned)nb, 256, 0, q>>>(pk, npix, g, ug, V, p_begin, p_end, 1,
                                                                             homs, out);
    } else if (vs) {
        if (ct) MPIV_U8(true, 4, true);
        else MPIV_U8(false, 4, true);
    } else if (ct) MPIV_U8(true, 2, false);
    else MPIV_U8(false, 2, false);
#undef MPIV_U8
    return launched(nm);
}

int mpiv_render_packed_u8(const uint32_t* packed, int H, int W, int P, const float* homs, int V, float* out,
                          void* stream) {
    return render_u8_impl(packed, H, W, P, 0, P, 1, homs, V, out, false, stream);
}

int mpiv_render_packed_u8_ct(const uint32_t* packed, int H, int W, int P, int p_begin, int p_end, int back,
                             const float* homs, int V, float* ct, void* stream) {
    return render_u8_impl(packed, H, W, P, p_begin, p_end, back, homs, V, ct, true, stream);
}

int mpiv_mark(int tag, void* stream) {
    if (tag < 1 || tag > 4096) return fail(MPIV_ERR_ARG, "mpiv_mark: tag must be in 1..4096");
    mark_kernel<<<tag, 64, 0, S(stream)>>>();
    return launched("mpiv_mark");
}

int mpiv_probe_gather(const float* window, size_t window_bytes, int iters, int blocks_, float* sink, void* stream) {
    if (!window || !sink) return fail(MPIV_ERR_ARG, "mpiv_probe_gather: null pointer");
    if (window_bytes < (size_t)kProbeWindow)
        return fail(MPIV_ERR_ARG, "mpiv_probe_gather: the window must hold >= %d bytes", (int)kProbeWindow);
    if (iters <= 0 || blocks_ <= 0) return fail(MPIV_ERR_ARG, "mpiv_probe_gather: bad size");
    if (!aligned16(window)) return fail(MPIV_ERR_ARG, "mpiv_probe_gather: window must be 16-byte aligned");
    probe_gather_kernel<<<blocks_, 256, 0, S(stream)>>>(reinterpret_cast<const float4*>(window), iters, sink);
    return launched("mpiv_probe_gather");
}

int mpiv_route(const char* entry, const int64_t* a, int na, char* name, int name_cap, int64_t* grid_threads) {
    if (!entry || !a || !name || name_cap <= 0) return fail(MPIV_ERR_ARG, "mpiv_route: null pointer");
    for (int i = 0; i < kNumOpts; ++i)
        if (opt((DebugOpt)i) != kOptDefaults[i])
            return fail(MPIV_ERR_ARG, "mpiv_route: reports the production routes only (debug options are set)");
    // nothing is dereferenced or launched in a dry run: any 256-B aligned address passes the checks
    alignas(256) static float dummy[64];
    float* d = dummy;
    RouteNote note{};
    int rc;
    g_route = &note;
    if (strcmp(entry, "render_packed") == 0 && na == 4)
        rc = render_packed_impl(d, (int)a[0], (int)a[1], (int)a[2], 0, (int)a[2], 1, d, (int)a[3], d, false, 0, nullptr);
    else if (strcmp(entry, "render_packed_ct") == 0 && na == 4)
        rc = render_packed_impl(d, (int)a[0], (int)a[1], (int)a[2], 0, (int)a[2], 1, d, (int)a[3], d, true, 0, nullptr);
    else if (strcmp(entry, "render_packed_ct_rows") == 0 && na == 6)
        rc = mpiv_render_packed_ct_rows(d, (int)a[0], (int)a[1], (int)a[2], 0, (int)a[2], 1, d, (int)a[3], (int)a[4],
                                        (int)a[5], d, nullptr);
    else if (strcmp(entry, "plane_sweep") == 0 && na == 7) {
        const int64_t C = a[3], D = a[4], st[4] = {a[1] * a[2] * C, a[2] * C, C, 1};
        rc = mpiv_plane_sweep(d, st, (int)a[0], (int)a[1], (int)a[2], (int)C, d, d, d, (int)D, (int)a[5], (int)a[6], d,
                              nullptr);
    } else if (strcmp(entry, "render_train") == 0 && na == 4) {
        const int64_t P = a[3], st[5] = {a[1] * a[2] * P * 4, a[2] * P * 4, P * 4, 4, 1};
        rc = mpiv_render_train(d, st, (int)a[0], (int)a[1], (int)a[2], (int)P, d, d, d, nullptr);
    } else if (strcmp(entry, "render_packed_u8") == 0 && na == 4) {
        rc = render_u8_impl(reinterpret_cast<const uint32_t*>(d), (int)a[0], (int)a[1], (int)a[2], 0, (int)a[2], 1, d,
                            (int)a[3], d, false, nullptr);
    } else if (strcmp(entry, "render_net_output") == 0 && na == 4) {
        const int64_t B = a[0], H = a[1], W = a[2], P = a[3];
        const int64_t ps[4] = {(2 * P + 3) * H * W, H * W, W, 1}, fs[4] = {H * W * 3, W * 3, 3, 1};
        rc = mpiv_render_net_output(d, ps, d, fs, (int)B, (int)H, (int)W, (int)P, d, d, nullptr);
    } else if (strcmp(entry, "render") == 0 && na == 4) {
        const int64_t P = a[3], st[5] = {a[1] * a[2] * P * 4, a[2] * P * 4, P * 4, 4, 1};
        rc = mpiv_render(d, st, (int)a[0], (int)a[1], (int)a[2], (int)P, d, d, nullptr);
    } else {
        g_route = nullptr;
        return fail(MPIV_ERR_ARG, "mpiv_route: unknown entry '%s' or wrong argument count %d", entry, na);
    }
    g_route = nullptr;
    if (rc != MPIV_OK) return rc;
    if (!note.name[0]) return fail(MPIV_ERR_ARG, "mpiv_route: '%s' has no reportable route", entry);
    snprintf(name, (size_t)name_cap, "%s", note.name);
    if (grid_threads) *grid_threads = note.threads;
    g_err[0] = '\0';
    return MPIV_OK;
}

// A/B diagnosis: the backward fallback's ticket protocol with trivial items (render_bwd.hip
// ticket_selftest_kernel).  ctr: 4 zeroed device words, marks: nphase * nvirt zeroed ints.
int mpiv_selftest_tickets(int blocks_, int nphase, int nvirt, unsigned poll_limit, unsigned* ctr, int* marks,
                          void* stream) {
#if MPIV_AB
    if (!ctr || !marks || blocks_ <= 0 || nphase <= 0 || nvirt <= 0) return fail(MPIV_ERR_ARG, "mpiv_selftest_tickets: bad args");
    ticket_selftest_kernel<<<blocks_, 256, 0, S(stream)>>>(ctr, marks, nphase, nvirt, poll_limit);
    return launched("mpiv_selftest_tickets");
#else
    (void)blocks_, (void)nphase, (void)nvirt, (void)poll_limit, (void)ctr, (void)marks, (void)stream;
    return fail(MPIV_ERR_ARG, "mpiv_selftest_tickets: an A/B diagnosis, built only into libmpiv_ab.so");
#endif
}

int mpiv_selftest_div_const(int divisor, unsigned long long* mismatches, void* stream) {
    if (!mismatches || divisor < 1) return fail(MPIV_ERR_ARG, "mpiv_selftest_div_const: bad args");
    const float c = (float)divisor;
    div_const_selftest_kernel<<<4096, 256, 0, S(stream)>>>(c, 1.0f / c, mismatches);
    return launched("mpiv_selftest_div_const");
}

}  // extern "C"
