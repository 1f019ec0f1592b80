// assemble.hip -- MPI assembly from the network output (the notebook's
// mpi_from_net_output, ipynb cell 10 L79-111) for gfx950.
//
// The network predicts, per pixel, P blend weights, P alphas and a background colour
// (channels-first [B, 2P+3, H, W], tanh domain); plane i of the MPI is
//     rgb_i   = w_i * fg + (1 - w_i) * bg,   w_i = (pred[i] + 1) / 2
//     alpha_i = (pred[P + i] + 1) / 2,        bg = pred[2P .. 2P+2],  fg = the reference image.
// The notebook builds this with a Python loop of P torch.cat calls (O(P^2) bytes
// copied); here one streaming pass writes the MPI either in the reference layout
// [B,H,W,P,4] (the drop-in's return value) or straight into the render's padded
// plane-major layout (mpiv_pack_planes'), so an inference render never materialises
// [B,H,W,P,4] at all.  Every value rounds like the notebook's ATen ops: add, the
// division by 2 (exact scaling, identical to * 0.5 for every input), mul, rsub, mul,
// add -- unfused (-ffp-contract=off).
//
// Backward (training: the notebook differentiates its loss through this assembly,
// ipynb cell 12 L5-15): d pred for the weights, alphas and background from
// d rgba [B,H,W,P,4], in autograd's order where it is defined -- per plane
// d w = (sum_c g_c*fg_c + -(sum_c g_c*bg_c)) / 2, d alpha = g_a / 2; the P background
// contributions g_c * (1 - w_i) accumulate from the last plane to the first.
// kZeroFlush: every d pred value ends with "+ 0.0f".  Autograd adds up the SliceBackward
// gradients of mpi_pred's three slices (weights, alphas, bg) and the SelectBackward ones of each
// plane, each zero-filled outside its slice, so every entry also receives +0 terms: a -0 (an
// all-zero d rgba, i.e. a texel no output pixel samples) becomes +0; every other value is
// unchanged (tests/golden/netout_train.npz).  d fg has no such slices and keeps its sign.
#include "mpiv_common.hpp"

namespace mpiv {

struct NetStrides {   // element strides
    int64_t pb, pc, py, px;   // pred [B, 2P+3, H, W]
    int64_t fb, fy, fx, fc;   // fg   [B, H, W, 3]
    int pred_bytes = 0, fg_bytes = 0;  // one batch element's byte span (0: not buffer-addressable)
};

// one MPI texel of plane p at pixel (y, x) of batch element b
__device__ __forceinline__ float4 assemble_texel(const float* __restrict__ pred, const float* __restrict__ fg,
                                                 const NetStrides& s, int P, int b, int p, int y, int x) {
    const float* pp = pred + (int64_t)b * s.pb + (int64_t)y * s.py + (int64_t)x * s.px;
    const float* fp = fg + (int64_t)b * s.fb + (int64_t)y * s.fy + (int64_t)x * s.fx;
    const float w = (pp[(int64_t)p * s.pc] + 1.0f) / 2.0f;         // blend weight
    const float a = (pp[(int64_t)(P + p) * s.pc] + 1.0f) / 2.0f;   // alpha
    const float om = 1.0f - w;
    float4 t;
    t.x = w * fp[0] + om * pp[(int64_t)(2 * P + 0) * s.pc];
    t.y = w * fp[s.fc] + om * pp[(int64_t)(2 * P + 1) * s.pc];
    t.z = w * fp[2 * s.fc] + om * pp[(int64_t)(2 * P + 2) * s.pc];
    t.w = a;
    return t;
}

// Reference layout out [B,H,W,P,4] (contiguous).  A block moves 64 pixels x 16 planes
// through LDS: the channel planes of pred are read along x (coalesced), the output
// leaves with the 16 planes of a pixel as one 256-B run.
constexpr int kAsmPix = 64;
constexpr int kAsmPl = 16;

// homs (mpiv_assemble_mpi_sampled, round 6): the render's [B][P][9] homographies; a block whose
// pixels lie outside every row its 16 planes' samples can read (render.hip sampled_rows, over the
// whole frame) writes nothing -- those texels of out keep whatever they held.
__global__ __launch_bounds__(256) void assemble_native_kernel(const float* __restrict__ pred,
                                                              const float* __restrict__ fg, NetStrides s, int H,
                                                              int W, int P, FastDiv w_div, float4* __restrict__ out,
                                                              const float* __restrict__ homs = nullptr,
                                                              RenderGeom g = RenderGeom{}) {
    __shared__ float4 tile[kAsmPl][kAsmPix + 1];
    const int64_t npix = (int64_t)H * W;
    const int64_t pix0 = (int64_t)blockIdx.x * kAsmPix;
    const int p0 = blockIdx.y * kAsmPl;
    const int b = blockIdx.z;
    if (homs) {
        const int ylo = (int)(pix0 / W), yhi = (int)(min(pix0 + kAsmPix, npix) - 1) / W;  // the block's rows
        bool need = false;
        if (threadIdx.x < kAsmPl && p0 + (int)threadIdx.x < P) {
            const int2 r = sampled_rows(homs + ((int64_t)b * P + p0 + threadIdx.x) * 9, 0.0f, (float)(W - 1), 0.0f,
                                        (float)(H - 1), g);
            need = r.x <= yhi && r.y >= ylo;
        }
        if (!__syncthreads_or(need)) return;
    }
    for (int k = threadIdx.x; k < kAsmPix * kAsmPl; k += blockDim.x) {  // pixel fastest
        const int i = k % kAsmPix, j = k / kAsmPix;
        const int64_t pix = pix0 + i;
        if (pix < npix && p0 + j < P) {
            const int y = (int)fast_div((unsigned)pix, w_div), x = (int)pix - y * W;
            tile[j][i] = assemble_texel(pred, fg, s, P, b, p0 + j, y, x);
        }
    }
    __syncthreads();
    for (int k = threadIdx.x; k < kAsmPix * kAsmPl; k += blockDim.x) {  // plane fastest
        const int j = k % kAsmPl, i = k / kAsmPl;
        const int64_t pix = pix0 + i;
        if (pix < npix && p0 + j < P) out[((int64_t)b * npix + pix) * P + p0 + j] = tile[j][i];
    }
}

// Padded plane-major layout of batch element b: packed [P][H+4][W+4] float4, 2-texel
// zero border (mpiv_pack_planes).  One work-item per padded texel of one plane.
__global__ __launch_bounds__(256) void assemble_packed_kernel(const float* __restrict__ pred,
                                                              const float* __restrict__ fg, NetStrides s, int H,
                                                              int W, int P, int b, FastDiv wp_div,
                                                              float4* __restrict__ packed, int64_t plane_stride) {
    const int64_t pix = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int p = blockIdx.y;
    if (pix >= plane_stride) return;
    const int yp = (int)fast_div((unsigned)pix, wp_div);
    const int y = yp - kPad, x = (int)pix - yp * (int)wp_div.d - kPad;
    float4 t = make_float4(0.f, 0.f, 0.f, 0.f);
    if ((unsigned)y < (unsigned)H && (unsigned)x < (unsigned)W) t = assemble_texel(pred, fg, s, P, b, p, y, x);
    packed[(int64_t)p * plane_stride + pix] = t;
}

// d pred [B, 2P+3, H, W] (contiguous) from d rgba [B,H,W,P,4] (strides gs[5]).
// One work-item per pixel walks the planes.
__global__ __launch_bounds__(256) void assemble_backward_kernel(const float* __restrict__ grad,
                                                                NativeStrides gs, const float* __restrict__ pred,
                                                                const float* __restrict__ fg, NetStrides s, int H,
                                                                int W, int P, FastDiv w_div,
                                                                float* __restrict__ dpred, float* __restrict__ dfg) {
    const int64_t npix = (int64_t)H * W;
    const int64_t pix = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int b = blockIdx.y;
    if (pix >= npix) return;
    const int y = (int)fast_div((unsigned)pix, w_div), x = (int)pix - y * W;
    const float* pp = pred + (int64_t)b * s.pb + (int64_t)y * s.py + (int64_t)x * s.px;
    const float* fp = fg + (int64_t)b * s.fb + (int64_t)y * s.fy + (int64_t)x * s.fx;
    const float f0 = fp[0], f1 = fp[s.fc], f2 = fp[2 * s.fc];
    const float b0 = pp[(int64_t)(2 * P) * s.pc], b1 = pp[(int64_t)(2 * P + 1) * s.pc],
                b2 = pp[(int64_t)(2 * P + 2) * s.pc];
    const float* g0 = grad + (int64_t)b * gs.b + (int64_t)y * gs.y + (int64_t)x * gs.x;
    float* dp = dpred + (int64_t)b * (2 * P + 3) * npix + pix;
    float db0 = 0.f, db1 = 0.f, db2 = 0.f, df0 = 0.f, df1 = 0.f, df2 = 0.f;
    for (int p = P - 1; p >= 0; --p) {  // autograd runs the planes' nodes last to first
        const float* g = g0 + (int64_t)p * gs.p;
        const float gr = g[0], gg = g[gs.c], gb = g[2 * gs.c], ga = g[3 * gs.c];
        const float w = (pp[(int64_t)p * s.pc] + 1.0f) / 2.0f;
        const float om = 1.0f - w;
        // MulBackward of w * fg (broadcast w: sum over the 3 channels) and of (1 - w) * bg
        const float sf = (gr * f0 + gg * f1) + gb * f2;
        const float sb = (gr * b0 + gg * b1) + gb * b2;
        const float dw = sf + -sb;  // RsubBackward negates; two terms commute exactly
        dp[(int64_t)p * npix] = dw / 2.0f + 0.0f;     // DivBackward; + 0: see kZeroFlush
        dp[(int64_t)(P + p) * npix] = ga / 2.0f + 0.0f;
        const float c0 = gr * om, c1 = gg * om, c2 = gb * om;
        const float e0 = gr * w, e1 = gg * w, e2 = gb * w;  // MulBackward of w * fg w.r.t. fg
        if (p == P - 1) {
            db0 = c0; db1 = c1; db2 = c2;
            df0 = e0; df1 = e1; df2 = e2;
        } else {
            db0 = db0 + c0; db1 = db1 + c1; db2 = db2 + c2;
            df0 = df0 + e0; df1 = df1 + e1; df2 = df2 + e2;
        }
    }
    dp[(int64_t)(2 * P) * npix] = db0 + 0.0f;
    dp[(int64_t)(2 * P + 1) * npix] = db1 + 0.0f;
    dp[(int64_t)(2 * P + 2) * npix] = db2 + 0.0f;
    if (dfg) {
        float* o = dfg + ((int64_t)b * npix + pix) * 3;
        o[0] = df0; o[1] = df1; o[2] = df2;
    }
}

// The same for a dense d rgba ([B,H,W,P,4] contiguous): 256 pixels per block; the
// gradient runs are staged through LDS 8 planes at a time (each pixel's 8 x 16 B read
// as one 128-B segment) instead of each lane walking its own P*16-B run.
constexpr int kAbPix = 256;
constexpr int kAbPl = 8;

__global__ __launch_bounds__(kAbPix) void assemble_backward_dense_kernel(const float4* __restrict__ grad,
                                                                        const float* __restrict__ pred,
                                                                        const float* __restrict__ fg, NetStrides s,
                                                                        int H, int W, int P, FastDiv w_div,
                                                                        float* __restrict__ dpred,
                                                                        float* __restrict__ dfg) {
    __shared__ float4 tile[kAbPix][kAbPl + 1];
    const int64_t npix = (int64_t)H * W;
    const int64_t pix0 = (int64_t)blockIdx.x * kAbPix;
    const int b = blockIdx.y;
    const int64_t pix = pix0 + threadIdx.x;
    const bool live = pix < npix;
    const int y = live ? (int)fast_div((unsigned)pix, w_div) : 0, x = live ? (int)pix - y * W : 0;
    const float* pp = pred + (int64_t)b * s.pb + (int64_t)y * s.py + (int64_t)x * s.px;
    const float* fp = fg + (int64_t)b * s.fb + (int64_t)y * s.fy + (int64_t)x * s.fx;
    float f0 = 0.f, f1 = 0.f, f2 = 0.f, b0 = 0.f, b1 = 0.f, b2 = 0.f;
    if (live) {
        f0 = fp[0]; f1 = fp[s.fc]; f2 = fp[2 * s.fc];
        b0 = pp[(int64_t)(2 * P) * s.pc]; b1 = pp[(int64_t)(2 * P + 1) * s.pc]; b2 = pp[(int64_t)(2 * P + 2) * s.pc];
    }
    const float4* gb = grad + (int64_t)b * npix * P;
    float* dp = dpred + (int64_t)b * (2 * P + 3) * npix + pix;
    float db0 = 0.f, db1 = 0.f, db2 = 0.f, df0 = 0.f, df1 = 0.f, df2 = 0.f;
    const int nch = (P + kAbPl - 1) / kAbPl;
    for (int ch = nch - 1; ch >= 0; --ch) {  // planes last to first, as autograd runs them
        const int p0 = ch * kAbPl, np = min(kAbPl, P - p0);
        __syncthreads();  // the previous chunk's reads of the tile are done
        for (int k = threadIdx.x; k < kAbPix * kAbPl; k += kAbPix) {
            const int i = k / kAbPl, j = k % kAbPl;
            if (pix0 + i < npix && j < np) tile[i][j] = gb[(pix0 + i) * P + p0 + j];
        }
        __syncthreads();
        if (!live) continue;
        for (int j = np - 1; j >= 0; --j) {
            const int p = p0 + j;
            const float4 g = tile[threadIdx.x][j];
            const float w = (pp[(int64_t)p * s.pc] + 1.0f) / 2.0f;
            const float om = 1.0f - w;
            const float sf = (g.x * f0 + g.y * f1) + g.z * f2;
            const float sb = (g.x * b0 + g.y * b1) + g.z * b2;
            dp[(int64_t)p * npix] = (sf + -sb) / 2.0f + 0.0f;
            dp[(int64_t)(P + p) * npix] = g.w / 2.0f + 0.0f;
            const float c0 = g.x * om, c1 = g.y * om, c2 = g.z * om;
            const float e0 = g.x * w, e1 = g.y * w, e2 = g.z * w;
            if (p == P - 1) {
                db0 = c0; db1 = c1; db2 = c2;
                df0 = e0; df1 = e1; df2 = e2;
            } else {
                db0 = db0 + c0; db1 = db1 + c1; db2 = db2 + c2;
                df0 = df0 + e0; df1 = df1 + e1; df2 = df2 + e2;
            }
        }
    }
    if (!live) return;
    dp[(int64_t)(2 * P) * npix] = db0 + 0.0f;
    dp[(int64_t)(2 * P + 1) * npix] = db1 + 0.0f;
    dp[(int64_t)(2 * P + 2) * npix] = db2 + 0.0f;
    if (dfg) {
        float* o = dfg + ((int64_t)b * npix + pix) * 3;
        o[0] = df0; o[1] = df1; o[2] = df2;
    }
}

// ---------------------------------------------------------------------------
// assembly fused into the render (inference / viewer: mpi_render_net_output_torch)
// ---------------------------------------------------------------------------
//
// One launch from the network output to the rendered views: a 512-thread block owns a
// 64x8 output tile of one view and walks the planes back to front; for each plane it
// assembles the texels of the tile's footprint box (render_lds.hip's box argument:
// corners through the exact recipe, one-texel margin, clipped to the 2-texel zero
// border) straight from pred / fg into LDS -- assemble_texel's exact arithmetic, zeros
// outside the image -- and the samples read their taps there.  The inputs of plane p+1's
// box are loaded into registers while plane p is sampled (one barrier per plane).  No
// MPI is written: per view the HBM traffic is the network output itself
// ((2P+3)*4 + 12 B per pixel) instead of that plus a packed MPI written and read back
// (P*16 B per pixel each way).  A sample whose tap origin is not staged, or a plane whose
// box does not fit, assembles its four taps directly (the same texel function), so the
// frame is bit-identical to assemble + render.
constexpr int kNTX = 64, kNTY = 8;
constexpr int kNThreads = kNTX * kNTY;
constexpr int kNCap = 1024;   // texels per staged box of a 64x8 tile (16 KiB)
constexpr int kNMaxP = 512;   // planes in the box table

// one texel of plane p at image texel (tx, ty), zero outside the image (grid_sample's
// zero padding of the packed border)
__device__ __forceinline__ float4 net_texel(const float* __restrict__ pred, const float* __restrict__ fg,
                                            const NetStrides& s, int H, int W, int P, int b, int p, int tx, int ty) {
    if ((unsigned)tx >= (unsigned)W || (unsigned)ty >= (unsigned)H) return make_float4(0.f, 0.f, 0.f, 0.f);
    return assemble_texel(pred, fg, s, P, b, p, ty, tx);
}

// raw inputs of one texel (w, alpha, bg, fg), loaded ahead of the assembly
struct NetRaw {
    float w, a, b0, b1, b2, f0, f1, f2;
    bool in;
};

__device__ __forceinline__ NetRaw net_load(const float* __restrict__ pred, const float* __restrict__ fg,
                                           const NetStrides& s, int H, int W, int P, int b, int p, int tx, int ty) {
    NetRaw r;
    r.in = (unsigned)tx < (unsigned)W && (unsigned)ty < (unsigned)H;
    const int cx = min(max(tx, 0), W - 1), cy = min(max(ty, 0), H - 1);  // always valid memory
    const float* pp = pred + (int64_t)b * s.pb + (int64_t)cy * s.py + (int64_t)cx * s.px;
    const float* fp = fg + (int64_t)b * s.fb + (int64_t)cy * s.fy + (int64_t)cx * s.fx;
    r.w = pp[(int64_t)p * s.pc];
    r.a = pp[(int64_t)(P + p) * s.pc];
    r.b0 = pp[(int64_t)(2 * P + 0) * s.pc];
    r.b1 = pp[(int64_t)(2 * P + 1) * s.pc];
    r.b2 = pp[(int64_t)(2 * P + 2) * s.pc];
    r.f0 = fp[0];
    r.f1 = fp[s.fc];
    r.f2 = fp[2 * s.fc];
    return r;
}

// assemble_texel's arithmetic on preloaded inputs (bit-identical)
__device__ __forceinline__ float4 net_assemble(const NetRaw& r) {
    if (!r.in) return make_float4(0.f, 0.f, 0.f, 0.f);
    const float w = (r.w + 1.0f) / 2.0f;
    const float a = (r.a + 1.0f) / 2.0f;
    const float om = 1.0f - w;
    float4 t;
    t.x = w * r.f0 + om * r.b0;
    t.y = w * r.f1 + om * r.b1;
    t.z = w * r.f2 + om * r.b2;
    t.w = a;
    return t;
}

// the same inputs split by lifetime: the plane's blend weight and alpha (w, a: from HBM, loaded
// DEPTH planes ahead) and the plane-independent background / reference colour (mostly cache hits:
// the neighbouring planes' boxes overlap, loaded one plane ahead)
struct NetWA {
    float w, a;
};
struct NetBF {
    float b0, b1, b2, f0, f1, f2;
    bool in;
};

__device__ __forceinline__ NetWA net_load_wa(const float* __restrict__ pred, const NetStrides& s, int H, int W, int P,
                                             int b, int p, int tx, int ty) {
    const int cx = min(max(tx, 0), W - 1), cy = min(max(ty, 0), H - 1);  // always valid memory
    const float* pp = pred + (int64_t)b * s.pb + (int64_t)cy * s.py + (int64_t)cx * s.px;
    return NetWA{pp[(int64_t)p * s.pc], pp[(int64_t)(P + p) * s.pc]};
}

__device__ __forceinline__ NetBF net_load_bf(const float* __restrict__ pred, const float* __restrict__ fg,
                                             const NetStrides& s, int H, int W, int P, int b, int tx, int ty) {
    NetBF r;
    r.in = (unsigned)tx < (unsigned)W && (unsigned)ty < (unsigned)H;
    const int cx = min(max(tx, 0), W - 1), cy = min(max(ty, 0), H - 1);
    const float* pp = pred + (int64_t)b * s.pb + (int64_t)cy * s.py + (int64_t)cx * s.px;
    const float* fp = fg + (int64_t)b * s.fb + (int64_t)cy * s.fy + (int64_t)cx * s.fx;
    r.b0 = pp[(int64_t)(2 * P + 0) * s.pc];
    r.b1 = pp[(int64_t)(2 * P + 1) * s.pc];
    r.b2 = pp[(int64_t)(2 * P + 2) * s.pc];
    r.f0 = fp[0];
    r.f1 = fp[s.fc];
    r.f2 = fp[2 * s.fc];
    return r;
}

// The same loads through buffer resources with 32-bit offsets (one batch element's spans < 2 GiB,
// render_netout_kernel<.., BUF = true>): a texel's address is one 32-bit offset shared by its
// loads, each channel plane / colour a scalar offset -- the 64-bit address arithmetic of the
// pointer loads was ~25 VALU per staged texel.
struct NetRsrc {
    __amdgpu_buffer_rsrc_t pred, fg;
    int pc4, fc4;  // channel strides in bytes
};

__device__ __forceinline__ NetWA net_load_wa_buf(const NetRsrc& r, const NetStrides& s, int H, int W, int P, int p,
                                                 int tx, int ty) {
    const int cx = min(max(tx, 0), W - 1), cy = min(max(ty, 0), H - 1);
    const int off = (cy * (int)s.py + cx * (int)s.px) * 4;
    return NetWA{llvm_raw_buffer_load_f32(r.pred, off, p * r.pc4, 0), llvm_raw_buffer_load_f32(r.pred, off, (P + p) * r.pc4, 0)};
}

// FG3 (round 6): the reference image's channels are contiguous (its [B,H,W,3] tensor as the notebook
// holds it), so a texel's colour is ONE 12-B load instead of three 4-B loads (6 load instructions
// per staged texel instead of 8).
template <bool FG3 = false>
__device__ __forceinline__ NetBF net_load_bf_buf(const NetRsrc& r, const NetStrides& s, int H, int W, int P, int tx,
                                                 int ty) {
    NetBF q;
    q.in = (unsigned)tx < (unsigned)W && (unsigned)ty < (unsigned)H;
    const int cx = min(max(tx, 0), W - 1), cy = min(max(ty, 0), H - 1);
    const int off = (cy * (int)s.py + cx * (int)s.px) * 4;
    const int offf = (cy * (int)s.fy + cx * (int)s.fx) * 4;
    q.b0 = llvm_raw_buffer_load_f32(r.pred, off, (2 * P) * r.pc4, 0);
    q.b1 = llvm_raw_buffer_load_f32(r.pred, off, (2 * P + 1) * r.pc4, 0);
    q.b2 = llvm_raw_buffer_load_f32(r.pred, off, (2 * P + 2) * r.pc4, 0);
    if (FG3) {
        const f32x3b f = llvm_raw_buffer_load_v3f32(r.fg, offf, 0, 0);
        q.f0 = f[0];
        q.f1 = f[1];
        q.f2 = f[2];
    } else {
        q.f0 = llvm_raw_buffer_load_f32(r.fg, offf, 0, 0);
        q.f1 = llvm_raw_buffer_load_f32(r.fg, offf, r.fc4, 0);
        q.f2 = llvm_raw_buffer_load_f32(r.fg, offf, 2 * r.fc4, 0);
    }
    return q;
}

__device__ __forceinline__ float4 net_assemble2(const NetWA& q, const NetBF& r) {
    return net_assemble(NetRaw{q.w, q.a, r.b0, r.b1, r.b2, r.f0, r.f1, r.f2, r.in});
}



// RPT rows per work-item: the block's tile is 64 x 8*RPT pixels (work-item (lane, wave) renders
// rows wave, wave + 8, ...), its staged box holds kNCap * RPT texels.  Taller tiles mean fewer
// blocks: at RPT = 2 a 1024x576 view is 576 blocks, all resident at once (3 per CU), where the
// 1152 blocks of RPT = 1 ran in two rounds of a latency-bound per-plane loop (round 4: 0.14 ms).
// NW waves per block (tile 64 x NW*RPT); the planes' w / a loads run DEPTH planes ahead (1: plane
// p+1's while plane p is sampled), bg / fg one plane ahead.
#ifndef MPIV_NET_EARLY
#define MPIV_NET_EARLY 1  // DB: the next plane's loads issued before the barrier
#endif
#ifndef MPIV_NET_BFONCE
#define MPIV_NET_BFONCE 0  // timing probe only (wrong frames): bg / fg loaded for plane 0's box alone
#endif
// DB (round 5): two staged boxes, plane p in buffer p & 1, so a plane needs one barrier (its box
// staged) instead of two -- the commit of plane p+1 goes to the other buffer, which plane p-1's
// samples finished reading before this plane's barrier.  The boxes get 100 texels per tile row
// (1600 at 64 x 16: the widest box of config 2's camera path is ~1570) and the box table sits in
// dynamic LDS sized by P, so 2 x 25.6 KiB keeps 3 blocks per CU.
template <int NW, int RPT, int DEPTH, bool BUF, bool DB = false, bool FG3 = false>
__global__ __launch_bounds__(64 * NW) void render_netout_kernel(const float* __restrict__ pred,
                                                                const float* __restrict__ fg, NetStrides ns,
                                                                RenderGeom g, int V, const float* __restrict__ homs,
                                                                float* __restrict__ out,
                                                                float4* __restrict__ ckpt = nullptr) {
    constexpr int kThreads = 64 * NW;
    constexpr int kTY = NW * RPT;
    constexpr int kCap = (DB ? 100 : 128) * kTY;  // texels per staged box: a 64 x 8 tile 1024 (its box at the
                                                  // swapped normalisation's x stretch 1.78: ~940; 64 x 16: up
                                                  // to ~1550)
    constexpr int kFill = (kCap + kThreads - 1) / kThreads;
    static_assert(DEPTH >= 1 && DEPTH <= 3, "planes in flight");
    __shared__ __attribute__((aligned(16))) float4 s_tex_all[DB ? 2 * kCap : kCap];
    extern __shared__ int2 s_box_dyn[];
    __shared__ int2 s_box_st[DB ? 1 : kNMaxP];  // per plane: (x_lo, y_lo), (rows, direct) as 16-bit pairs
    int2* s_box = DB ? s_box_dyn : s_box_st;
    __shared__ int s_pitch;
    const int tiles_x = (g.W + kNTX - 1) / kNTX;
    const int lb = xcd_logical_block(blockIdx.x, gridDim.x);
    const int v = lb % V;
    const int tile = lb / V;
    const int tx0 = (tile % tiles_x) * kNTX, ty0 = (tile / tiles_x) * kTY;
    const int lane = threadIdx.x & (kWave - 1), wave = threadIdx.x >> 6;
    const int x = tx0 + lane;
    const float* hv = homs + (int64_t)v * g.P * 9;
    const int P = g.P;
    if (threadIdx.x == 0) s_pitch = 0;
    __syncthreads();
    // ---- footprint boxes (thread q -> plane q/4, corner q%4) + the tile's division proof
    const int cx1 = min(tx0 + kNTX - 1, g.W - 1), cy1 = min(ty0 + kTY - 1, g.H - 1);
    bool ok_div = true, dead = true;
    for (int q0 = 0; q0 < 4 * P; q0 += kThreads) {
        const int q = q0 + (int)threadIdx.x;
        const bool live = q < 4 * P;
        const int pl = live ? (q >> 2) : 0;
        const int corner = q & 3;
        const float fx = (float)((corner & 1) ? cx1 : tx0), fy = (float)((corner & 2) ? cy1 : ty0);
        const float* h = hv + (int64_t)pl * 9;
        if (live && corner == 0) {
            const bool safe = div2_rect_safe(h, (float)tx0, (float)cx1, (float)ty0, (float)cy1);
            ok_div = ok_div && safe;
            dead = dead && safe && tile_dead(h, (float)tx0, (float)cx1, (float)ty0, (float)cy1, g);
        }
        float px, py;
        render_pos<true>(h, fx, fy, g, px, py);
        float w = __builtin_fmaf(h[7], fy, h[6] * fx) + h[8];
        w = (w == 0.0f) ? w + 1e-8f : w;
        const bool fin = __builtin_isfinite(px) && __builtin_isfinite(py) && __builtin_fabsf(px) < 1e7f &&
                         __builtin_fabsf(py) < 1e7f;
        float xmin = floorf(px), xmax = xmin, ymin = floorf(py), ymax = ymin;
        int pos = fin && w > 0.0f, neg = fin && w < 0.0f;
#pragma unroll
        for (int m = 1; m <= 2; m <<= 1) {
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
            const int direct = (!ok || width < 2 || rows < 2 || width > 256 || width * rows > kCap) ? 1 : 0;
            s_box[q >> 2] = make_int2((xl & 0xFFFF) | (yl << 16), rows | (direct << 16));
            if (!direct) atomicMax(&s_pitch, width);
        }
    }
    const bool proven = __syncthreads_and(ok_div);
    if (__syncthreads_and(dead)) {  // every plane samples the zero border over the whole tile (render.hip tile_dead)
        for (int r = 0; r < RPT; ++r) {
            const int y = ty0 + wave + NW * r;
            if (x >= g.W || y >= g.H) continue;
            float cr = -0.0f, cg = -0.0f, cb = -0.0f, t = 1.0f;
            for (int p = 0; p < P; ++p) {
                composite_zero<false>(p, p + 1, p == 0, cr, cg, cb, t);
                if (ckpt && (p & 7) == 7 && p + 1 < P)
                    ckpt[(((int64_t)v * ((P + 7) >> 3) + ((p + 1) >> 3)) * g.H + y) * g.W + x] =
                        make_float4(cr, cg, cb, 0.0f);
            }
            const int64_t o = (((int64_t)v * g.H + y) * g.W + x) * 3;
            out[o + 0] = cr;
            out[o + 1] = cg;
            out[o + 2] = cb;
        }
        return;
    }
    const int pitch = s_pitch;
    auto box_of = [&](int i) {
        const int2 bb = s_box[i];
        return make_int4((int)(short)(bb.x & 0xFFFF), bb.x >> 16, bb.y & 0xFFFF, bb.y >> 16);
    };
    auto staged = [&](const int4& bx) { return bx.w == 0 && bx.z * pitch <= kCap; };
    // this thread's box texels: idx = tid + 512*j -> (row, col) with the common pitch
    int row_j[kFill], col_j[kFill];
#pragma unroll
    for (int j = 0; j < kFill; ++j) {
        const int idx = (int)threadIdx.x + kThreads * j;
        row_j[j] = pitch > 0 ? idx / pitch : 0;
        col_j[j] = idx - row_j[j] * pitch;
    }
    NetWA wa[DEPTH][kFill];
    NetBF bf[kFill];
    NetRsrc rs;
    if (BUF) {
        rs.pred = make_rsrc(pred + (int64_t)v * ns.pb, ns.pred_bytes);
        rs.fg = make_rsrc(fg + (int64_t)v * ns.fb, ns.fg_bytes);
        rs.pc4 = (int)ns.pc * 4;
        rs.fc4 = (int)ns.fc * 4;
    }
    auto fetch_wa = [&](NetWA (&st)[kFill], int p, const int4& bx) {
        const int nfp = bx.z * pitch;
#pragma unroll
        for (int j = 0; j < kFill; ++j)
            if (kThreads * j < nfp)  // block-uniform
                st[j] = BUF ? net_load_wa_buf(rs, ns, g.H, g.W, P, p, bx.x + col_j[j], bx.y + row_j[j])
                            : net_load_wa(pred, ns, g.H, g.W, P, v, p, bx.x + col_j[j], bx.y + row_j[j]);
    };
    auto fetch_bf = [&](const int4& bx) {
        const int nfp = bx.z * pitch;
#pragma unroll
        for (int j = 0; j < kFill; ++j)
            if (kThreads * j < nfp)
                bf[j] = BUF ? net_load_bf_buf<FG3>(rs, ns, g.H, g.W, P, bx.x + col_j[j], bx.y + row_j[j])
                            : net_load_bf(pred, fg, ns, g.H, g.W, P, v, bx.x + col_j[j], bx.y + row_j[j]);
    };
    auto commit = [&](const NetWA (&st)[kFill], const int4& bx, float4* s_tex) {
        const int nfp = bx.z * pitch;
#pragma unroll
        for (int j = 0; j < kFill; ++j)
            if ((int)threadIdx.x + kThreads * j < nfp) s_tex[threadIdx.x + kThreads * j] = net_assemble2(st[j], bf[j]);
    };
    const float fx = (float)x;
    float cr[RPT], cg[RPT], cb[RPT];
#pragma unroll
    for (int r = 0; r < RPT; ++r) cr[r] = cg[r] = cb[r] = -0.0f;  // plane 0 replaces it exactly (render.hip)
    auto sample = [&](int p, const int4& bx, const float4* s_tex) {
        const float* hp = hv + (int64_t)p * 9;
#pragma unroll
        for (int r = 0; r < RPT; ++r) {
            const int y = ty0 + wave + NW * r;
            if (x < g.W && y < g.H) {
                const float fy = (float)y;
                float px, py;
                if (proven)
                    render_pos_fast<false>(hp, fx, fy, g, px, py);
                else
                    render_pos<true>(hp, fx, fy, g, px, py);
                TapSet ts;
                bool hit = false;
                if (staged(bx)) {
                    const LdsBox box = make_lds_box(bx.x, bx.y, bx.z, pitch, g.W, g.H);
                    hit = lds_issue(s_tex, box, px, py, ts);
                }
                if (!hit) {  // assemble the four taps directly (rare)
                    const float fx0 = floorf(px), fy0 = floorf(py);
                    const float wx = px - fx0, ex = 1.0f - wx;
                    const float wy = py - fy0, sy = 1.0f - wy;
                    ts.nw = sy * ex;
                    ts.ne = sy * wx;
                    ts.sw = wy * ex;
                    ts.se = wy * wx;
                    const int ix = (int)__builtin_amdgcn_fmed3f(fx0, -2.0f, (float)g.W);
                    const int iy = (int)__builtin_amdgcn_fmed3f(fy0, -2.0f, (float)g.H);
                    const float4 t0 = net_texel(pred, fg, ns, g.H, g.W, P, v, p, ix, iy);
                    const float4 t1 = net_texel(pred, fg, ns, g.H, g.W, P, v, p, ix + 1, iy);
                    const float4 t2 = net_texel(pred, fg, ns, g.H, g.W, P, v, p, ix, iy + 1);
                    const float4 t3 = net_texel(pred, fg, ns, g.H, g.W, P, v, p, ix + 1, iy + 1);
                    ts.a = {t0.x, t0.y, t0.z, t0.w};
                    ts.b = {t1.x, t1.y, t1.z, t1.w};
                    ts.c = {t2.x, t2.y, t2.z, t2.w};
                    ts.d = {t3.x, t3.y, t3.z, t3.w};
                }
                const f32x4 sm = blend_taps(ts);
                const float a = p == 0 ? 1.0f : sm[3];
                const float om = 1.0f - a;
                cr[r] = over(sm[0], a, om, cr[r]);
                cg[r] = over(sm[1], a, om, cg[r]);
                cb[r] = over(sm[2], a, om, cb[r]);
                // training forward: the colour before every 8-plane chunk c >= 1, render_train's
                // [V][ceil(P/8)][H][W] checkpoints (the backward's chain rebuilds each chunk from it)
                if (ckpt && (p & 7) == 7 && p + 1 < P)
                    ckpt[(((int64_t)v * ((P + 7) >> 3) + ((p + 1) >> 3)) * g.H + y) * g.W + x] =
                        make_float4(cr[r], cg[r], cb[r], 0.0f);
            }
        }
    };
    // plane p: its w / a (fetched DEPTH planes earlier into ring slot p % DEPTH) and bg / fg (fetched
    // one plane earlier) are assembled into LDS; then the slot takes plane p + DEPTH's w / a and bf
    // plane p + 1's bg / fg, in flight while plane p is sampled
    auto step = [&](int p, NetWA (&st)[kFill]) {
        const int4 bx = box_of(p);
        float4* s_tex = s_tex_all + (DB ? (p & 1) * kCap : 0);
        if (staged(bx)) commit(st, bx, s_tex);
        auto fetch_next = [&]() {
            if (p + 1 < P && !MPIV_NET_BFONCE) {
                const int4 bn = box_of(p + 1);
                if (staged(bn)) fetch_bf(bn);
            }
            if (p + DEPTH < P) {
                const int4 bn = box_of(p + DEPTH);
                if (staged(bn)) fetch_wa(st, p + DEPTH, bn);
            }
        };
        if (DB && MPIV_NET_EARLY) fetch_next();  // the registers are free once committed: load before the barrier
        __syncthreads();  // plane p's box is in LDS (DB: and plane p-1's samples are done with the other buffer)
        if (!(DB && MPIV_NET_EARLY)) fetch_next();
        sample(p, bx, s_tex);
        if (!DB) __syncthreads();  // every sample of plane p has read the box
    };
    if (staged(box_of(0))) fetch_bf(box_of(0));
#pragma unroll
    for (int d = 0; d < DEPTH; ++d)
        if (d < P && staged(box_of(d))) fetch_wa(wa[d], d, box_of(d));
    int p = 0;
    for (; p + DEPTH <= P; p += DEPTH) {
#pragma unroll
        for (int d = 0; d < DEPTH; ++d) step(p + d, wa[d]);  // static ring slots
    }
#pragma unroll
    for (int d = 0; d < DEPTH; ++d)
        if (p + d < P) step(p + d, wa[d]);
#pragma unroll
    for (int r = 0; r < RPT; ++r) {
        const int y = ty0 + wave + NW * r;
        if (x < g.W && y < g.H) {
            const int64_t o = (((int64_t)v * g.H + y) * g.W + x) * 3;
            out[o + 0] = cr[r];
            out[o + 1] = cg[r];
            out[o + 2] = cb[r];
        }
    }
}

}  // namespace mpiv
