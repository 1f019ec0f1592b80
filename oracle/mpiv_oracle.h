/* mpiv_oracle.h -- CPU restatement of the reference arithmetic (TEST INFRASTRUCTURE ONLY).
 * See mpiv_oracle.c for the per-step citations into the reference utils.py.
 * All strides are in ELEMENTS (floats). */
#ifndef MPIV_ORACLE_H
#define MPIV_ORACLE_H
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif
/* mpi [B,H,W,P,4] with strides st[5]; homs [B][P][9] row-major; out [B,H,W,3] contiguous */
void oracle_render(const float *mpi, const int64_t st[5], int B, int H, int W, int P,
                   const float *homs, float *out, int nthreads);
/* plane-range partial (C,T) [B,H,W,4] of planes [p0,p1); back: range holds plane 0 */
void oracle_render_ct(const float *mpi, const int64_t st[5], int B, int H, int W, int P, int p0, int p1,
                      int back, const float *homs, float *out, int nthreads);
/* img [B,Hs,Ws,C] strides st[4]; ki [B][9]; proj [B][16]; depths [D] fp32; out [B,Ht,Wt,D*C] */
void oracle_plane_sweep(const float *img, const int64_t st[4], int B, int Hs, int Ws, int C,
                        const float *ki, const float *proj, const float *depths, int D,
                        int Ht, int Wt, float *out, int nthreads);
/* in [N,C,Hi,Wi] strides ist; coords [N,Ho,Wo,2] contiguous (in [0,1] units); out strides ost (N,C,H,W) */
void oracle_grid_sample(const float *in, const int64_t ist[4], int N, int C, int Hi, int Wi,
                        const float *coords, int Ho, int Wo, float *out, const int64_t ost[4],
                        int nthreads);
/* d(render)/d(mpi) like the reference's autograd: dout [B,H,W,3] contiguous ->
 * dmpi [B,H,W,P,4] contiguous (overwritten); vec = grid_sampler's Vec<float> width */
void oracle_render_backward(const float *mpi, const int64_t st[5], int B, int H, int W, int P,
                            const float *homs, const float *dout, float *dmpi, int vec, int nthreads);
/* layers [P][n][4] contiguous; out [n][3] */
void oracle_over_composite(const float *layers, int P, int64_t n, float *out);
/* depth-map inverse warp: img [B,Hs,Ws,C] (strides), ki [B][9], proj [B][16],
 * depth [B][Ht][Wt] contiguous -> out [B,Ht,Wt,C] */
void oracle_inverse_warp(const float *img, const int64_t st[4], int B, int Hs, int Ws, int C,
                         const float *ki, const float *proj, const float *depth, int Ht, int Wt,
                         float *out, int nthreads);
/* counter-based synthetic MPI (synth.hip restated): planes [p0,p1) as [H][W][p1-p0][4] */
void oracle_synth_mpi(uint32_t seed, int H, int W, int p0, int p1, float *out);
/* rows [y0,y1) of one view of the synthetic MPI through planes [p0,p1), homs [P][9]:
 * ct = 0 -> final render [y1-y0][W][3]; ct = 1 -> (C,T) partial [y1-y0][W][4] */
void oracle_render_synth(uint32_t seed, int H, int W, int P, int p0, int p1, int back, int ct,
                         const float *homs, int y0, int y1, float *out, int nthreads);
#ifdef __cplusplus
}
#endif
#endif
