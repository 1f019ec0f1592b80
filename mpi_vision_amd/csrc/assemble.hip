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
#include "mpiv_common.hpp"

namespace mpiv {

struct NetStrides {   // element strides
    int64_t pb, pc, py, px;   // pred [B, 2P+3, H, W]
    int64_t fb, fy, fx, fc;   // fg   [B, H, W, 3]
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

__global__ __launch_bounds__(256) void assemble_native_kernel(const float* __restrict__ pred,
                                                              const float* __restrict__ fg, NetStrides s, int H,
                                                              int W, int P, FastDiv w_div, float4* __restrict__ out) {
    __shared__ float4 tile[kAsmPl][kAsmPix + 1];
    const int64_t npix = (int64_t)H * W;
    const int64_t pix0 = (int64_t)blockIdx.x * kAsmPix;
    const int p0 = blockIdx.y * kAsmPl;
    const int b = blockIdx.z;
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
        dp[(int64_t)p * npix] = dw / 2.0f;            // DivBackward
        dp[(int64_t)(P + p) * npix] = ga / 2.0f;
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
    dp[(int64_t)(2 * P) * npix] = db0;
    dp[(int64_t)(2 * P + 1) * npix] = db1;
    dp[(int64_t)(2 * P + 2) * npix] = db2;
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
            dp[(int64_t)p * npix] = (sf + -sb) / 2.0f;
            dp[(int64_t)(P + p) * npix] = g.w / 2.0f;
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
    dp[(int64_t)(2 * P) * npix] = db0;
    dp[(int64_t)(2 * P + 1) * npix] = db1;
    dp[(int64_t)(2 * P + 2) * npix] = db2;
    if (dfg) {
        float* o = dfg + ((int64_t)b * npix + pix) * 3;
        o[0] = df0; o[1] = df1; o[2] = df2;
    }
}

}  // namespace mpiv
