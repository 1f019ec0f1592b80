// mpiv_common.hpp -- device-side arithmetic shared by the MPI render / plane-sweep
// kernels (gfx950, wave64).
//
// Every helper rounds exactly like the ATen CPU ops the reference utils.py runs
// (SURVEY.md §8a recipe; pinned bit-exact by tests/test_oracle.py against the
// reference's own outputs).  The library is compiled with -ffp-contract=off, so an
// FMA appears only where it is written as __builtin_fmaf.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace mpiv {

constexpr int kWave = 64;

typedef float f32x4 __attribute__((ext_vector_type(4)));

// 16-byte raw buffer load.  ROCm 7.2's __builtin_amdgcn_raw_buffer_load_b128 lowers to
// a 4-byte buffer_load_dword (observed in the .s; the other 12 bytes are garbage), so
// the LLVM intrinsic is bound directly, as composable_kernel does.
__device__ f32x4 llvm_raw_buffer_load_v4f32(__amdgpu_buffer_rsrc_t rsrc, int voffset, int soffset,
                                            int aux) __asm("llvm.amdgcn.raw.ptr.buffer.load.v4f32");
__device__ float llvm_raw_buffer_load_f32(__amdgpu_buffer_rsrc_t rsrc, int voffset, int soffset,
                                          int aux) __asm("llvm.amdgcn.raw.ptr.buffer.load.f32");

// Out-of-range buffer offset: the buffer unit's range check returns 0 for it without
// touching memory -- exactly grid_sample's per-tap zero padding.
constexpr int kOOB = 0x7FFFFF00;

__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* base, int bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, bytes, 0x00020000);
}

// Exact unsigned division n / d by a launch-constant d >= 1 for n < 2^31
// (Granlund-Montgomery: q = (mulhi(n, m) + n) >> s with m = floor(2^32 (2^s - d) / d) + 1,
// s = ceil(log2 d)); replaces the ~40-instruction 64-bit division in index math.
struct FastDiv {
    unsigned d, m;
    int s;
};

inline FastDiv make_fastdiv(unsigned d) {
    FastDiv f;
    f.d = d;
    int s = 0;
    while ((1ull << s) < d) ++s;
    f.s = s;
    f.m = (unsigned)((((1ull << 32) * ((1ull << s) - d)) / d) + 1);
    return f;
}

__host__ __device__ __forceinline__ unsigned fast_div(unsigned n, const FastDiv& f) {
#ifdef __HIP_DEVICE_COMPILE__
    const unsigned t = __umulhi(n, f.m);
#else
    const unsigned t = (unsigned)(((unsigned long long)n * f.m) >> 32);
#endif
    return (t + n) >> f.s;
}

// Correctly rounded fp32 division.  hipcc's default expansion of `a / b` is the
// IEEE-exact v_div_scale / v_rcp / fma / v_div_fmas / v_div_fixup sequence; it is
// kept verbatim (a reciprocal-multiply shifts coordinates by 1 ulp -> ~1e-4 output
// error on sharp texels, measured in the survey).
__device__ __forceinline__ float div_rn(float a, float b) { return a / b; }

// Correctly rounded x / c for a launch-uniform divisor c >= 1, given rc = RN(1/c)
// (computed on the host as 1.0f / c): q = RN(x*rc) is faithful, its residual
// r = fma(-c, q, x) is exact, and one correction fma(r, rc, q) then rounds to RN(x/c)
// (Markstein's theorem for a correctly rounded reciprocal).  v_div_scale / v_div_fixup
// are not needed: they only act when |x| or the quotient leaves the normal range, and
// there (|x / c| < 2^-26, or x = +-inf) the quotient cannot change the sample position:
// -1 + 2*cx rounds to -1 for any |cx| < 2^-26, and an infinite coordinate yields NaN
// weights either way.  Checked against IEEE division for all 2^32 inputs and the
// divisors of tests/test_render_gpu.py::test_div_const_exhaustive.  3 VALU instead of 11.
__device__ __forceinline__ float div_const(float x, float c, float rc) {
    const float q = x * rc;
    const float r = __builtin_fmaf(-c, q, x);
    return __builtin_fmaf(r, rc, q);
}

// Correctly rounded u / w and v / w sharing one reciprocal.  This is hipcc's IEEE
// division sequence (v_rcp + one Newton step, q = a*y, two residual corrections;
// the last is what v_div_fmas computes) without v_div_scale / v_div_fixup, which are
// identities unless an operand or the quotient leaves the normal range.  The guard
// keeps the fast path where they are identities for every quotient that can move a
// sample position (|q| >= 2^-26: smaller quotients round -1 + 2q/(H-1) to -1
// regardless); anything else takes the plain IEEE division.
__device__ __forceinline__ float div_core(float a, float b, float y) {
    float q = a * y;
    float r = __builtin_fmaf(-b, q, a);
    q = __builtin_fmaf(r, y, q);
    r = __builtin_fmaf(-b, q, a);
    return __builtin_fmaf(r, y, q);
}

__device__ __forceinline__ bool div2_safe(float u, float v, float w) {
    const float aw = __builtin_fabsf(w);
    return aw >= 0x1p-60f && aw <= 0x1p60f && __builtin_fmaxf(__builtin_fabsf(u), __builtin_fabsf(v)) <= 0x1p60f;
}

__device__ __forceinline__ void div2_rn(float u, float v, float w, float& qu, float& qv) {
    if (__builtin_expect(div2_safe(u, v, w), 1)) {
        float y = __builtin_amdgcn_rcpf(w);
        const float e = __builtin_fmaf(-w, y, 1.0f);
        y = __builtin_fmaf(e, y, y);
        qu = div_core(u, w, y);
        qv = div_core(v, w, y);
    } else {
        qu = div_rn(u, w);
        qv = div_rn(v, w);
    }
}

// div2_rn's fast path alone (valid for every lane where div2_safe holds).  Kernels that
// keep several samples in flight run it for all of them and patch the rare unsafe lanes
// afterwards, so the common path has no branch between the samples.
__device__ __forceinline__ void div2_fast(float u, float v, float w, float& qu, float& qv) {
    float y = __builtin_amdgcn_rcpf(w);
    const float e = __builtin_fmaf(-w, y, 1.0f);
    y = __builtin_fmaf(e, y, y);
    qu = div_core(u, w, y);
    qv = div_core(v, w, y);
}

// divide_safe_torch (utils.py:35-39) fused with div2_rn: w == 0 -> w + 1e-8, then u/w, v/w.
// The guard lives in the rare branch only: w == 0 fails div2_safe.
__device__ __forceinline__ void divide_safe2(float u, float v, float w, float& qu, float& qv) {
    if (__builtin_expect(div2_safe(u, v, w), 1)) {
        float y = __builtin_amdgcn_rcpf(w);
        const float e = __builtin_fmaf(-w, y, 1.0f);
        y = __builtin_fmaf(e, y, y);
        qu = div_core(u, w, y);
        qv = div_core(v, w, y);
    } else {
        w = (w == 0.0f) ? w + 1e-8f : w;  // utils.py:38
        qu = div_rn(u, w);
        qv = div_rn(v, w);
    }
}

// grid value g in [-1, 1] -> source pixel, align_corners=False (ATen CPU vectorised
// grid sampler: (g + 1) * (size / 2) - 0.5, contracted to one FMA).
__device__ __forceinline__ float unnormalize(float g, float half_size) {
    return __builtin_fmaf(g + 1.0f, half_size, -0.5f);
}

// -1 + 2*c (utils.py:127, :406).  2*c is exact, so one FMA rounds identically.
__device__ __forceinline__ float to_grid(float c) { return __builtin_fmaf(2.0f, c, -1.0f); }

// Bilinear weights + per-tap in-bounds flags for one sample point.
struct Bilinear {
    float nw, ne, sw, se;
    int ix, iy;                  // floor(px), floor(py) as ints (valid where the flags say)
    bool x0, x1, y0, y1;         // tap column/row inside the image
};

__device__ __forceinline__ Bilinear bilinear_setup(float px, float py, int Wi, int Hi) {
    Bilinear b;
    const float fx0 = floorf(px), fy0 = floorf(py);
    const float w = px - fx0, e = 1.0f - w;
    const float n = py - fy0, s = 1.0f - n;
    b.nw = s * e;
    b.ne = s * w;
    b.sw = n * e;
    b.se = n * w;
    // float compares: NaN / huge coordinates are simply out of bounds (== ATen's int
    // compares for every finite coordinate)
    b.x0 = (fx0 >= 0.0f) & (fx0 < (float)Wi);
    b.x1 = (fx0 >= -1.0f) & (fx0 < (float)(Wi - 1));
    b.y0 = (fy0 >= 0.0f) & (fy0 < (float)Hi);
    b.y1 = (fy0 >= -1.0f) & (fy0 < (float)(Hi - 1));
    // clamp before the int conversion so the index is always defined
    b.ix = (int)fminf(fmaxf(fx0, -1.0f), (float)Wi);
    b.iy = (int)fminf(fmaxf(fy0, -1.0f), (float)Hi);
    return b;
}

// v = nw_v*nw; v = fma(ne_v, ne, v); v = fma(sw_v, sw, v); v = fma(se_v, se, v)
__device__ __forceinline__ float blend4(const Bilinear& b, float v_nw, float v_ne, float v_sw, float v_se) {
    float acc = v_nw * b.nw;
    acc = __builtin_fmaf(v_ne, b.ne, acc);
    acc = __builtin_fmaf(v_sw, b.sw, acc);
    acc = __builtin_fmaf(v_se, b.se, acc);
    return acc;
}

// Over operator, back-to-front, unfused like the reference's separate tensor ops
// (utils.py:155-156): out = rgb*a + out*(1-a).
__device__ __forceinline__ float over(float rgb, float a, float one_minus_a, float out) {
    const float t0 = rgb * a;
    const float t2 = out * one_minus_a;
    return t0 + t2;
}

// Target pixel (x, y) through a row-major 3x3 homography -> normalised sample
// position (px, py) in source pixels, the render's recipe (utils.py:178-188, 127;
// grid_sample unnormalise).  inv_hm1 / inv_wm1 are NOT reciprocals: the reference
// divides by (H-1) and (W-1), so those stay true divisions.
__device__ __forceinline__ void hom_sample_pos(const float* __restrict__ h, float fx, float fy,
                                               float hm1, float wm1, float half_w, float half_h,
                                               float& px, float& py) {
    const float u = __builtin_fmaf(h[1], fy, h[0] * fx) + h[2];
    const float v = __builtin_fmaf(h[4], fy, h[3] * fx) + h[5];
    float w = __builtin_fmaf(h[7], fy, h[6] * fx) + h[8];
    w = (w == 0.0f) ? w + 1e-8f : w;  // divide_safe_torch, utils.py:38
    const float cx = div_rn(div_rn(u, w), hm1);  // SWAPPED: x / (H-1), utils.py:188
    const float cy = div_rn(div_rn(v, w), wm1);  //          y / (W-1)
    px = unnormalize(to_grid(cx), half_w);
    py = unnormalize(to_grid(cy), half_h);
}

// ---------------------------------------------------------------------------
// 16-B texel gathers from a plane of float4 texels through a buffer resource
// ---------------------------------------------------------------------------

// One bilinear sample in flight: the four 16-B taps (already issued) + weights.
struct TapSet {
    f32x4 a, b, c, d;           // NW, NE, SW, SE texels (0 where outside the plane)
    float nw, ne, sw, se;
};

// Issue the four tap loads of one sample of one packed plane.  Taps outside the
// plane (and every tap when `live` is false) get the out-of-range offset, so the
// buffer unit returns 0 for them without a memory access: grid_sample's zeros
// padding, per tap.
__device__ __forceinline__ void issue_taps(__amdgpu_buffer_rsrc_t r, int W, int H, float px, float py, bool live,
                                           TapSet& t) {
    const float fx0 = floorf(px), fy0 = floorf(py);
    const float wx = px - fx0, ex = 1.0f - wx;
    const float wy = py - fy0, sy = 1.0f - wy;
    t.nw = sy * ex;
    t.ne = sy * wx;
    t.sw = wy * ex;
    t.se = wy * wx;
    // clamp to [-2, W] / [-2, H] so the int conversion is defined and every tap index
    // outside [0, W) / [0, H) stays outside; unsigned compares then test the range
    const unsigned ux = (unsigned)(int)__builtin_amdgcn_fmed3f(fx0, -2.0f, (float)W);
    const unsigned uy = (unsigned)(int)__builtin_amdgcn_fmed3f(fy0, -2.0f, (float)H);
    const unsigned uw = (unsigned)W, uh = (unsigned)H;
    // signed 24-bit multiply (full rate): iy in [-2, H] and W < 2^23; iy = -1 must stay
    // negative because the south taps of that row are valid
    const int off = __mul24((int)uy, W) * 16 + (int)ux * 16;
    const int off_s = off + W * 16;
    // the +16 of the east taps is applied after the select so it folds into the
    // instruction's immediate offset; kOOB - 16 + 16 is still out of range
    t.a = llvm_raw_buffer_load_v4f32(r, (live && ux < uw && uy < uh) ? off : kOOB, 0, 0);
    t.b = llvm_raw_buffer_load_v4f32(r, ((live && ux + 1 < uw && uy < uh) ? off : kOOB - 16) + 16, 0, 0);
    t.c = llvm_raw_buffer_load_v4f32(r, (live && ux < uw && uy + 1 < uh) ? off_s : kOOB, 0, 0);
    t.d = llvm_raw_buffer_load_v4f32(r, ((live && ux + 1 < uw && uy + 1 < uh) ? off_s : kOOB - 16) + 16, 0, 0);
}

// Packed planes carry a kPad-texel zero border: plane p is [(H + 4)][(W + 4)] float4 and
// image texel (x, y) sits at ((y + 2) * Wp + x + 2), Wp = W + 4.  Clamping floor(px) into
// [-2, W] and floor(py) into [-2, H] keeps every tap of a sample inside the padded plane,
// and a clamped tap lands in the border exactly when the true tap is outside the image
// (both taps of an axis are outside whenever the clamp moved it), so the zeros padding
// of grid_sample needs no per-tap test: 6 VALU of address math for the four taps.
constexpr int kPad = 2;

// org = byte offset of image texel (0, 0) in the padded plane; row = Wp * 16.
__device__ __forceinline__ void issue_taps_padded(__amdgpu_buffer_rsrc_t r, int W, int H, int Wp, int org,
                                                  int row, float px, float py, TapSet& t) {
    const float fx0 = floorf(px), fy0 = floorf(py);
    const float wx = px - fx0, ex = 1.0f - wx;
    const float wy = py - fy0, sy = 1.0f - wy;
    t.nw = sy * ex;
    t.ne = sy * wx;
    t.sw = wy * ex;
    t.se = wy * wx;
    // med3 also maps NaN to a bound, so the index is always defined (the NaN weights
    // still make the sample NaN, as in the reference)
    const int cx = (int)__builtin_amdgcn_fmed3f(fx0, -2.0f, (float)W);
    const int cy = (int)__builtin_amdgcn_fmed3f(fy0, -2.0f, (float)H);
    const int off = (__mul24(cy, Wp) + cx) * 16 + org;  // >= 0, < plane bytes
    t.a = llvm_raw_buffer_load_v4f32(r, off, 0, 0);
    t.b = llvm_raw_buffer_load_v4f32(r, off + 16, 0, 0);
    t.c = llvm_raw_buffer_load_v4f32(r, off, row, 0);
    t.d = llvm_raw_buffer_load_v4f32(r, off + 16, row, 0);
}

__device__ __forceinline__ f32x4 blend_taps(const TapSet& t) {
    f32x4 o;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        float acc = t.a[k] * t.nw;
        acc = __builtin_fmaf(t.b[k], t.ne, acc);
        acc = __builtin_fmaf(t.c[k], t.sw, acc);
        acc = __builtin_fmaf(t.d[k], t.se, acc);
        o[k] = acc;
    }
    return o;
}

// ---------------------------------------------------------------------------
// bilinear taps from a footprint staged in LDS (render_mv.hip, sweep.hip)
// ---------------------------------------------------------------------------

// A staged box holds `rows` rows of `pitch` consecutive texels of a padded plane whose
// first texel is image texel (xl, yl) (xl, yl >= -2; the last staged row is <= H+1).
// A tap origin (floor px, floor py) is read from LDS at offsets (x0 - xl, y0 - yl)
// clamped to [0, xspan] x [0, yspan]: both of its columns and rows are staged and
// neither column lies past the padded row end W+1 (staged texels beyond it belong to
// the next padded row), xspan = min(xl + pitch - 2, W) - xl, yspan = rows - 2.
// The read is exact when the origin needed no clamp, and also when it was clamped
// onto a box edge that is the padded plane's border (-2, or W / H for the last
// origin): then both the clamped and the true taps lie outside the image, where the
// border's zeros are exactly grid_sample's zero padding (issue_taps_padded clamps the
// same way).  Any other origin is not staged.
struct LdsBox {
    float xl, yl;        // box origin (image texel coordinates)
    float xspan, yspan;  // largest tap-origin offsets served from LDS
    float gxl, gxh;      // tap-origin x offsets read exactly: [0, xspan], open at border edges
    float gyl, gyh;
    int pitch;           // staged row pitch (texels)
};

__device__ __forceinline__ LdsBox make_lds_box(int xl, int yl, int rows, int pitch, int W, int H) {
    LdsBox b;
    const int xspan = min(xl + pitch - 2, W) - xl, yspan = rows - 2;
    b.xl = (float)xl;
    b.yl = (float)yl;
    b.xspan = (float)xspan;
    b.yspan = (float)yspan;
    b.gxl = xl == -2 ? -__builtin_inff() : 0.0f;
    b.gxh = xl + xspan == W ? __builtin_inff() : b.xspan;
    b.gyl = yl == -2 ? -__builtin_inff() : 0.0f;
    b.gyh = yl + yspan == H ? __builtin_inff() : b.yspan;
    b.pitch = pitch;
    return b;
}

// First half of lds_sample: the weights and the four tap reads (in flight on return).
__device__ __forceinline__ bool lds_issue(const float4* __restrict__ tex, const LdsBox& b, float px, float py,
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
    const float4* st = tex + (int)__builtin_fmaf(iy, (float)b.pitch, ix);  // < rows * pitch: exact
    t.a = *reinterpret_cast<const f32x4*>(st);
    t.b = *reinterpret_cast<const f32x4*>(st + 1);
    t.c = *reinterpret_cast<const f32x4*>(st + b.pitch);
    t.d = *reinterpret_cast<const f32x4*>(st + b.pitch + 1);
    return (__builtin_amdgcn_fmed3f(rx, b.gxl, b.gxh) == rx) & (__builtin_amdgcn_fmed3f(ry, b.gyl, b.gyh) == ry);
}

// lds_issue for C = 3 texels: the tap reads are ds_read_b96 (the padding channel is
// never read), 12 VGPRs per tap instead of 16.
typedef float f32x3 __attribute__((ext_vector_type(3)));
struct TapSet3 {
    f32x3 a, b, c, d;
    float nw, ne, sw, se;
};

__device__ __forceinline__ bool lds_issue3(const float4* __restrict__ tex, const LdsBox& b, float px, float py,
                                           TapSet3& t) {
    const float fx0 = floorf(px), fy0 = floorf(py);
    const float wx = px - fx0, ex = 1.0f - wx;
    const float wy = py - fy0, sy = 1.0f - wy;
    t.nw = sy * ex;
    t.ne = sy * wx;
    t.sw = wy * ex;
    t.se = wy * wx;
    const float rx = fx0 - b.xl, ry = fy0 - b.yl;
    const float ix = __builtin_amdgcn_fmed3f(rx, 0.0f, b.xspan);
    const float iy = __builtin_amdgcn_fmed3f(ry, 0.0f, b.yspan);
    const float4* st = tex + (int)__builtin_fmaf(iy, (float)b.pitch, ix);
    t.a = *reinterpret_cast<const f32x3*>(st);
    t.b = *reinterpret_cast<const f32x3*>(st + 1);
    t.c = *reinterpret_cast<const f32x3*>(st + b.pitch);
    t.d = *reinterpret_cast<const f32x3*>(st + b.pitch + 1);
    return (__builtin_amdgcn_fmed3f(rx, b.gxl, b.gxh) == rx) & (__builtin_amdgcn_fmed3f(ry, b.gyl, b.gyh) == ry);
}

__device__ __forceinline__ f32x4 blend_taps3(const TapSet3& t) {
    f32x4 o;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        float acc = t.a[k] * t.nw;
        acc = __builtin_fmaf(t.b[k], t.ne, acc);
        acc = __builtin_fmaf(t.c[k], t.sw, acc);
        acc = __builtin_fmaf(t.d[k], t.se, acc);
        o[k] = acc;
    }
    o[3] = 0.0f;
    return o;
}

// One bilinear sample from the staged box, with the weights and fma chain of
// issue_taps_padded + blend_taps.  Returns false when the tap origin is not staged
// (see LdsBox; NaN included): its result is then meaningless and the caller gathers
// that sample from global memory instead -- so a staged kernel is bit-identical to the
// direct one whatever the box covers.
__device__ __forceinline__ bool lds_sample(const float4* __restrict__ tex, const LdsBox& b, float px, float py,
                                           f32x4& s) {
    TapSet t;
    const bool ok = lds_issue(tex, b, px, py, t);
    s = blend_taps(t);
    return ok;
}

}  // namespace mpiv
