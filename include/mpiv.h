/*
 * mpiv.h -- C ABI of libmpiv.so, the MI355X (gfx950) kernels behind the
 * mpi-vision hot path.
 *
 * The reference (Findeton/mpi-vision) has no FFI layer: its hot path is the
 * Python module functions of utils.py.  Each entry point below replaces the
 * per-pixel work of the reference function cited next to it; the Python
 * drop-in (mpi_vision_amd/utils.py) binds them with ctypes.
 *
 * Conventions
 *  - Every pointer is DEVICE memory owned by the caller (e.g. a torch tensor);
 *    the library never allocates or frees on these paths.
 *  - Strides are in ELEMENTS (floats), int64.  A stride may be 0 (broadcast).
 *  - `stream` is a hipStream_t (NULL = default stream).  Calls are
 *    stream-ordered and asynchronous; the library keeps no mutable global state
 *    (re-entrant, safe from several streams / threads).
 *  - Return 0 on success, a negative MPIV_ERR_* code otherwise; the message is
 *    available from mpiv_last_error() on the calling thread.  Never aborts.
 *  - All arithmetic is fp32 and rounds exactly like the reference's ATen CPU
 *    ops; matrices (homographies, Ki, proj) are computed by the
 *    caller on the host and passed as device buffers.
 */
#ifndef MPIV_H
#define MPIV_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MPIV_ABI_VERSION 14

enum {
    MPIV_OK = 0,
    MPIV_ERR_ARG = -1,   /* bad shape / stride / alignment / null pointer */
    MPIV_ERR_HIP = -2,   /* a HIP runtime call or kernel launch failed */
};

int mpiv_abi_version(void);
const char *mpiv_last_error(void);

/* First 16 hex digits of the sha256 of the sources the library was built from
 * (mpi_vision_amd/csrc/SOURCES, in order); the Python binding refuses a library
 * whose id does not match the sources next to it (a stale build). */
const char *mpiv_build_id(void);

/* Debug / A/B hook, never needed in production: selects a non-default kernel variant
 * by name ("render_mv", "render_pair", "render_native_lds", "render_chunk", "render_ring",
 * "render_tile", "render_vshare", "chunk_rows", "chunk_flight", "sweep_tile", "sweep_store",
 * "sweep_dlane", "sweep_rows", "sweep_direct", "box_shrink", "bwd_fallback", "bwd_margin",
 * "bwd_gather", "bwd_poll_limit", "bwd_fb_blocks", "bwd_fb_mode", "chunk_strip", "u8_flight", "bwd_group",
 * "netout_geo", "netout_buf", "bwd_overlap", "sweep_band", "sweep_pf", "sweep_soa"; "reset" restores every
 * default; abi.hip documents the values).  Values that
 * select a kernel kept only for A/B measurement return MPIV_ERR_ARG from libmpiv.so (they are
 * compiled into libmpiv_ab.so).  Process-wide; returns MPIV_ERR_ARG for an unknown name. */
int mpiv_debug_set(const char *name, int value);

/* Dry run of an entry point's production dispatch (no device memory touched, nothing
 * launched): writes the name of the kernel the call WOULD launch (as it appears in
 * rocprofv3's kernel names, template arguments included) into name[name_cap] and its grid
 * size in work-items into *grid_threads (may be NULL).  bench.py uses it to find its
 * launches in rocprofv3 summaries.  entry / args:
 *   "render_packed", "render_packed_ct"  {H, W, P, V}        (mpiv_render_packed[_ct])
 *   "render"                             {B, H, W, P}        (mpiv_render, contiguous MPI)
 *   "plane_sweep"                        {B, Hs, Ws, C, D, Ht, Wt} (mpiv_plane_sweep)
 *   "render_packed_ct_rows"              {H, W, P, V, y_begin, y_end} (mpiv_render_packed_ct_rows)
 *   "render_packed_u8"                   {H, W, P, V}        (mpiv_render_packed_u8)
 *   "render_net_output"                  {B, H, W, P}        (mpiv_render_net_output)
 * Fails while a debug option is set (it reports production routes only). */
int mpiv_route(const char *entry, const int64_t *args, int nargs, char *name, int name_cap, int64_t *grid_threads);

/* ---- MPI render -------------------------------------------------------- */

/* mpi_render_view_torch (utils.py:267-294), fused warp + over-composite.
 * mpi:   [B,H,W,P,4] with element strides mpi_strides[5] (B may be stride 0)
 * homs:  [B][P][9] row-major target->source homographies
 *        (inv_homography_torch, utils.py:44-67, evaluated by the caller)
 * out:   [B,H,W,3] contiguous
 * Planes contiguous per pixel (strides[3] == 4, strides[4] == 1, 16-B texels) are read
 * in place at full-line coalescing (render_chunk.hip); other layouts by a per-pixel
 * gather kernel. */
int mpiv_render(const float *mpi, const int64_t mpi_strides[5], int B, int H, int W, int P,
                const float *homs, float *out, void *stream);

/* mpiv_render for training (the forward of RenderFunction when rgba_layers needs a
 * gradient): the same frames, bit for bit, from the in-place chunked kernel, plus the
 * composited colour before every 8-plane chunk, ckpt [B][ceil(P/8)][H][W] float4 (16-B
 * aligned; chunk 0's slot is unused), which mpiv_render_backward takes instead of
 * recomputing the forward composite.  Needs the in-place layout (16-B texels, planes
 * contiguous per pixel, strides[3] == 4, strides[4] == 1), H, W >= 2 and P <= 796. */
int mpiv_render_train(const float *mpi, const int64_t mpi_strides[5], int B, int H, int W, int P,
                      const float *homs, float *out, float *ckpt, void *stream);

/* Layout pack for repeated rendering of one MPI: one view [H,W,P,4] (element
 * strides strides[4] = H,W,P,C) -> plane-major packed [P][H+4][W+4][4] (16-B
 * aligned, contiguous) with a 2-texel zero border around every plane; image texel
 * (x, y) of plane p is packed[p][y+2][x+2].  The border is grid_sample's zero
 * padding made explicit, so the render kernels need no per-tap range test.  No
 * reference counterpart (the reference re-materialises a plane-major copy on every
 * call, utils.py:121). */
int mpiv_pack_planes(const float *mpi_view, const int64_t strides[4], int H, int W, int P,
                     float *packed, void *stream);

/* mpi_render_view_torch on a packed MPI (mpiv_pack_planes layout) for V views at once.
 * homs [V][P][9]; out [V,H,W,3] contiguous.  Direct bilinear gathers, blocks ordered so
 * the views of one output tile share an XCD's L2 (render.hip). */
int mpiv_render_packed(const float *packed, int H, int W, int P, const float *homs, int V,
                       float *out, void *stream);

/* mpiv_render_packed through the counting build of render_rows_kernel (same frames): adds to
 * *census (device, caller-zeroed) the number of 64-lane 16-B gather instructions the launch
 * issues -- the texture path's real work, which vertical tap reuse makes smaller than 4 per
 * plane-sample (bench.py's roofline).  Fails unless the launch routes to the rows kernel. */
int mpiv_render_packed_census(const float *packed, int H, int W, int P, const float *homs, int V, float *out,
                              unsigned long long *census, void *stream);

/* The same with the LDS-staged kernel (per-tile plane footprints staged by LDS-DMA):
 * identical output; kept for A/B measurement. */
int mpiv_render_packed_lds(const float *packed, int H, int W, int P, const float *homs, int V,
                           float *out, void *stream);

/* Plane-range partial for plane sharding: planes [p_begin, p_end)
 * of a packed MPI -> ct [V,H,W,4] = (C rgb, T).  back != 0: the range holds the
 * reference's plane 0 (its alpha ignored, utils.py:152-153) -> T = 0. */
int mpiv_render_packed_ct(const float *packed, int H, int W, int P, int p_begin, int p_end, int back,
                          const float *homs, int V, float *ct, void *stream);

/* Rows [y_begin, y_end) of mpiv_render_packed_ct's partial (same bits; the other rows of ct
 * [V,H,W,4] are not written): the plane-sharded render launches its row bands one at a time so
 * each band's exchange overlaps the next band's render.  H, W >= 2. */
int mpiv_render_packed_ct_rows(const float *packed, int H, int W, int P, int p_begin, int p_end, int back,
                               const float *homs, int V, int y_begin, int y_end, float *ct, void *stream);

/* Ordered over-operator combine: parts [G][n][4] (C,T), index 0 = back-most range
 * -> out [n][3].  (Cf,Tf) o (Cb,Tb) = (Cf + Tf*Cb, Tf*Tb). */
int mpiv_combine_ct(const float *parts, int G, int64_t n, float *out, void *stream);

/* HOST function (no device memory): the per-(view, plane) target->source homographies
 * of mpi_render_view_torch (utils.py:278-285 -> 255-262 -> 225-229 -> inv_homography_torch
 * 44-67), bit-identical to the reference's torch-CPU fp32 chain.
 * pose [B][4][4], depths [P] (plane depths, far->near), K and Kinv = inverse(K) [B][3][3]
 * (host, row-major) -> H [B][P][9]. */
int mpiv_render_homographies(const float *pose, const float *depths, const float *K, const float *Kinv, int B,
                             int P, float *H);

/* The same chain evaluated on the device (all five pointers DEVICE memory), one
 * work-item per (view, plane): bit-identical to mpiv_render_homographies, for callers
 * whose poses and intrinsics live in HBM (no blocking device-to-host copies). */
int mpiv_render_homographies_device(const float *pose, const float *depths, const float *K, const float *Kinv,
                                    int B, int P, float *H, void *stream);

/* HOST function: proj = [[K_src, 0], [0, 0, 0, 1]] @ pose [B][4][4] for the plane sweep /
 * inverse warp (projective_inverse_warp_torch[2], utils.py:428-438, 747-757: the torch.cat
 * of the padded K, then torch.matmul), bit-identical to the reference's torch-CPU fp32 ops.
 * Ks: [B][3][3] at batch stride ks_bstride floats (0: one K for every pose). */
int mpiv_psv_proj(const float *Ks, int64_t ks_bstride, const float *pose, int B, float *proj);

/* The same on the device (Ks, pose, proj in device memory), bit-identical to the host
 * entry: the PSV drop-ins use it when the pose already lives in HBM. */
int mpiv_psv_proj_device(const float *Ks, int64_t ks_bstride, const float *pose, int B, float *proj, void *stream);

/* ---- render backward ------------------------------------------------------ */

/* Workspace bytes for the fastest schedule of mpiv_render_backward on one H x W x P MPI
 * (reused across views): 16 B per plane-pixel of d samples for every plane + 2 B per
 * plane-pixel of colour checkpoints + the fallback's bucket arrays (<= 16 B per plane-pixel
 * of one plane group, groups sized to at most 2^25 plane-pixels).  Config 4: 3.0 GB. */
size_t mpiv_render_backward_workspace_size(int H, int W, int P);

/* The smallest workspace (round 4): given less than the size above, mpiv_render_backward runs
 * a view in plane groups of <= 2^25 plane-pixels, back to front, holding one group's d samples
 * at a time (bit-identical gradients, a few percent slower).  Config 4: 1.3 GB. */
size_t mpiv_render_backward_workspace_size_min(int H, int W, int P);

/* d(mpi_render_view_torch)/d(rgba_layers) (utils.py:267-294 under autograd), bit-exact
 * to the reference's CPU autograd: the over-composite adjoint followed by
 * grid_sampler_2d_backward's scatter, summed per texel in ATen's order.
 * mpi:     the forward's [V,H,W,P,4] rgba_layers IN PLACE, element strides mpi_strides[5]
 *          with 16-byte aligned texels and planes contiguous per pixel (strides[3] == 4,
 *          strides[4] == 1; a stride-0 broadcast batch is fine); any P (more than 796 planes
 *          read their homographies from global memory instead of LDS);
 * homs:    [V][P][9] (the forward's); dout: [V,H,W,3] contiguous incoming gradient;
 * ckpt:    NULL, or the checkpoints mpiv_render_train wrote in the forward of these views
 *          (then the adjoint skips recomputing the forward composite);
 * dmpi:    [V,H,W,P,4] contiguous, 16-byte aligned: view v's gradient is written (not
 *          accumulated);
 * workspace: >= mpiv_render_backward_workspace_size(H, W, P) bytes, 256-B aligned.
 * Deterministic (no float atomics); H*W < 2^26, P*H*W < 2^31.
 * A view the tile gather cannot prove complete runs the bucket fallback, whose phases are
 * ordered by tickets (no block needs to be resident: safe beside other streams, RCCL kernels
 * and other processes).  If a fallback wait ever outlasts its poll limit (not expected), that
 * view's gradient is NaN-filled and counted; mpiv_render_backward_status reports the count. */
int mpiv_render_backward(const float *mpi, const int64_t mpi_strides[5], int V, int H, int W, int P,
                         const float *homs, const float *dout, const float *ckpt, float *dmpi,
                         void *workspace, size_t workspace_bytes, void *stream);

/* mpiv_render_backward that also reports an aborted view without a copy: the calling process's abort
 * flag of the current device (mpiv_render_backward_abort_flag) is set to 1 -- a device store into a
 * page-locked, device-mapped int, visible to the host without a copy -- when a view's bucket fallback
 * aborted and its gradient was NaN-filled.  The caller reads and clears the flag on the host (the
 * Python layer does so before every default backward, so a training loop fails at the latest one
 * step after an abort, with no per-call copy, event or synchronisation). */
int mpiv_render_backward_watched(const float *mpi, const int64_t mpi_strides[5], int V, int H, int W, int P,
                                 const float *homs, const float *dout, const float *ckpt, float *dmpi,
                                 void *workspace, size_t workspace_bytes, void *stream);

/* The calling process's abort flag of device `device` (a page-locked int mapped into every device,
 * fine-grained, allocated on first use).  NULL if the allocation failed or device is out of [0, 64). */
int *mpiv_render_backward_abort_flag(int device);

/* Views of the last mpiv_render_backward call on this workspace (same H, W, P) whose
 * fallback aborted -> *aborted_views.  SYNCHRONISES the stream (the one entry point that
 * does): a checker for tests and debug runs, not for the training loop. */
int mpiv_render_backward_status(const void *workspace, int H, int W, int P, int *aborted_views, void *stream);

/* ---- MPI assembly from the network output ------------------------------- */

/* mpi_from_net_output (fast-torch-stereo-vision.ipynb cell 10 L79-111): the network's
 * channels-first prediction pred [B, 2P+3, H, W] (element strides pred_strides[4];
 * channels 0..P-1 blend weights, P..2P-1 alphas, 2P..2P+2 background rgb, tanh domain)
 * and the reference image fg [B,H,W,3] (fg_strides[4]) -> the MPI
 *   rgba[b,y,x,p] = (w*fg + (1-w)*bg, (pred[P+p]+1)/2),  w = (pred[p]+1)/2,
 * rounded like the notebook's ATen ops (bit-exact).  rgba: [B,H,W,P,4] contiguous,
 * 16-B aligned. */
int mpiv_assemble_mpi(const float *pred, const int64_t pred_strides[4], const float *fg,
                      const int64_t fg_strides[4], int B, int H, int W, int P, float *rgba, void *stream);

/* mpiv_assemble_mpi for the backward of a render of the assembled MPI (the fused net-output
 * training's re-assembly, round 6): homs [B][P][9] are that render's homographies; texel rows
 * no output pixel's in-image taps can read (exact bounds of the sample positions over the
 * frame, one row of margin; every row where they cannot be proven) are left UNWRITTEN.  Only
 * for mpiv_render_backward of those homographies. */
int mpiv_assemble_mpi_sampled(const float *pred, const int64_t pred_strides[4], const float *fg,
                              const int64_t fg_strides[4], int B, int H, int W, int P, const float *homs,
                              float *rgba, void *stream);

/* The same for batch element b, written straight into the render's packed layout
 * (mpiv_pack_planes: [P][H+4][W+4][4] with a zero border): assembly + pack in one
 * pass, no [B,H,W,P,4] tensor. */
int mpiv_assemble_mpi_packed(const float *pred, const int64_t pred_strides[4], const float *fg,
                             const int64_t fg_strides[4], int b, int H, int W, int P, float *packed,
                             void *stream);

/* mpi_render_view_torch(mpi_from_net_output(pred, fg), ...) in ONE kernel (inference /
 * viewer path): homs [B][P][9] (the render's homographies, view b renders batch element
 * b's MPI); out [B,H,W,3] contiguous.  Each plane's tile footprint is assembled from
 * pred / fg straight into LDS; no MPI tensor is written.  Bit-identical to
 * mpiv_assemble_mpi followed by mpiv_render.  2 <= H, W < 32764, P <= 512. */
int mpiv_render_net_output(const float *pred, const int64_t pred_strides[4], const float *fg,
                           const int64_t fg_strides[4], int B, int H, int W, int P, const float *homs, float *out,
                           void *stream);

/* The same kernel as the TRAINING forward of the fused path (mpi_render_net_output_torch under
 * autograd; the reference trains through mpi_from_net_output -> mpi_render_view_torch,
 * ipynb cell 12 L7-11 / L38-42): frames as mpiv_render_net_output, plus the composite
 * checkpoints ckpt [B][ceil(P/8)][H][W][4] that mpiv_render_train writes for the same MPI
 * (colour before every 8-plane chunk c >= 1; slot 0 unused) -- bit-identical to them, so
 * mpiv_render_backward can take them for the assembled MPI.  ckpt 16-B aligned. */
int mpiv_render_net_output_train(const float *pred, const int64_t pred_strides[4], const float *fg,
                                 const int64_t fg_strides[4], int B, int H, int W, int P, const float *homs,
                                 float *out, float *ckpt, void *stream);

/* Backward of mpiv_assemble_mpi (the notebook trains through it, cell 12 L5-15):
 * drgba [B,H,W,P,4] (drgba_strides[5]) -> dpred [B,2P+3,H,W] contiguous and, when dfg is
 * not NULL, d fg [B,H,W,3] contiguous (both written, not accumulated).  Per plane
 * dw = (sum_c g*fg - sum_c g*bg)/2, dalpha = g_a/2; d bg = sum over planes (last to
 * first) of g*(1-w); d fg = the same sum of g*w (autograd's order, bit-exact). */
int mpiv_assemble_mpi_backward(const float *drgba, const int64_t drgba_strides[5], const float *pred,
                               const int64_t pred_strides[4], const float *fg, const int64_t fg_strides[4],
                               int B, int H, int W, int P, float *dpred, float *dfg, void *stream);

/* ---- plane sweep -------------------------------------------------------- */

/* plane_sweep_torch / plane_sweep_torch_one / plane_sweep_torch_one2
 * (utils.py:452-471, 513-533, 771-799).
 * img:    [B,Hs,Ws,C] element strides img_strides[4]
 * ki:     [B][9]  inverse(tgt intrinsics)         (utils.py:370 / :747)
 * proj:   [B][16] [[K_src,0],[0,0,0,1]] @ pose     (utils.py:431-438 / :750-757)
 * depths: [D] fp32
 * out:    [B,Ht,Wt,D*C] contiguous, channel d*C + c (torch.cat order, utils.py:470)
 * C <= 4 reads img in place: D <= 2 by plane_sweep_direct_kernel (taps gathered per sample),
 * 3 <= D <= 8 by plane_sweep_px_kernel (pixel per lane, taps gathered per sample, the wave's
 * samples stored as one run), more depths by plane_sweep_dlane_kernel (the tile's source
 * footprint staged in LDS); C > 4 by the generic one-sample-per-thread kernel.  Every route
 * writes the same bits. */
int mpiv_plane_sweep(const float *img, const int64_t img_strides[4], int B, int Hs, int Ws, int C,
                     const float *ki, const float *proj, const float *depths, int D, int Ht, int Wt,
                     float *out, void *stream);

/* mpiv_plane_sweep with proj formed on the device from a pose in HBM (the notebook's dataset
 * call): proj_scratch [B][16] receives [[K_src, 0], [0, 0, 0, 1]] @ pose (mpiv_psv_proj_device,
 * bit-identical to the reference's torch-CPU proj), then the sweep runs from it.  Ks [B][3][3]
 * at batch stride ks_bstride floats (0: one camera), pose [B][4][4]; ki as mpiv_plane_sweep. */
int mpiv_plane_sweep_pose(const float *img, const int64_t img_strides[4], int B, int Hs, int Ws, int C,
                          const float *ki, const float *Ks, int64_t ks_bstride, const float *pose,
                          float *proj_scratch, const float *depths, int D, int Ht, int Wt, float *out,
                          void *stream);

/* The same writing into a wider tensor (C <= 4): element (b, pixel, d, c) goes to
 * out[b*out_bstride + pixel*out_pstride + d*C + c] (format_network_input_torch, utils.py:473-498,
 * writes each source's volume at its channel offset of the concatenated network input);
 * out_pstride >= D*C.  mpiv_plane_sweep with C <= 4 is this call with the dense strides. */
int mpiv_plane_sweep_into(const float *img, const int64_t img_strides[4], int B, int Hs, int Ws, int C,
                          const float *ki, const float *proj, const float *depths, int D, int Ht, int Wt,
                          float *out, int64_t out_bstride, int64_t out_pstride, void *stream);

/* Source images for the fast sweep: [B,Hs,Ws,C] (C <= 4, element strides) ->
 * img4 [B][Hs+4][Ws+4] 16-B texels (channels >= C zero) with a 2-texel zero border
 * (the packed-plane convention of mpiv_pack_planes), 16-B aligned. */
int mpiv_pad_texels(const float *img, const int64_t img_strides[4], int B, int Hs, int Ws, int C, float *img4,
                    void *stream);

/* plane_sweep_torch* on padded texels (mpiv_pad_texels), C <= 4, (Hs+4)*(Ws+4)*16 < 2 GiB:
 * same contract and bit-identical output as mpiv_plane_sweep. */
int mpiv_plane_sweep_padded(const float *img4, int B, int Hs, int Ws, int C, const float *ki, const float *proj,
                            const float *depths, int D, int Ht, int Wt, float *out, void *stream);

/* The same, writing into a wider tensor: element (b, pixel, d, c) goes to
 * out[b*out_bstride + pixel*out_pstride + d*C + c] (format_network_input_torch,
 * utils.py:473-498, writes each source's volume at its channel offset of the
 * concatenated network input).  out_pstride >= D*C. */
int mpiv_plane_sweep_padded_into(const float *img4, int B, int Hs, int Ws, int C, const float *ki,
                                 const float *proj, const float *depths, int D, int Ht, int Wt, float *out,
                                 int64_t out_bstride, int64_t out_pstride, void *stream);

/* projective_inverse_warp_torch / projective_inverse_warp_torch2 with a per-pixel
 * depth map (utils.py:409-450, 725-769).
 * depth: [B,Ht,Wt] element strides depth_strides[3]; out [B,Ht,Wt,C] contiguous. */
int mpiv_inverse_warp(const float *img, const int64_t img_strides[4], int B, int Hs, int Ws, int C,
                      const float *ki, const float *proj, const float *depth, const int64_t depth_strides[3],
                      int Ht, int Wt, float *out, void *stream);

/* ---- sampling / compositing primitives ---------------------------------- */

/* bilinear_wrapper_torch (utils.py:104-134) / resampler_wrapper_torch
 * (utils.py:395-407): grid_sample(bilinear, zeros, align_corners=False) at
 * -1 + 2*coords.
 * in:     [N,C,Hi,Wi] element strides in_strides[4]
 * coords: [N,Ho,Wo,2] element strides coord_strides[4] (last = component stride)
 * out:    element strides out_strides[4] in (N,C,H,W) order (NCHW or NHWC memory) */
int mpiv_grid_sample(const float *in, const int64_t in_strides[4], int N, int C, int Hi, int Wi,
                     const float *coords, const int64_t coord_strides[4], int Ho, int Wo, float *out,
                     const int64_t out_strides[4], void *stream);

/* over_composite (utils.py:136-157).
 * layers: DEVICE array of P pointers, each to n RGBA pixels with element strides
 *         (pixel_stride, channel_stride); layer 0 is the back.  out [n][3]. */
int mpiv_over_composite(const float *const *layers, int P, int64_t n, int64_t pixel_stride,
                        int64_t channel_stride, float *out, void *stream);

/* ---- geometry helpers ---------------------------------------------------- */

/* transform_points_torch (utils.py:69-88): pts [M][n][3], homs [M][9] -> out [M][n][3] */
int mpiv_transform_points(const float *pts, int M, int64_t n, const float *homs, float *out, void *stream);

/* normalize_homogeneous_torch (utils.py:90-101): pts [n][k+1] -> out [n][k];
 * w == 0 is replaced by 1e-8 IN pts, as the reference's in-place `+=` does. */
int mpiv_normalize_homogeneous(float *pts, int64_t n, int k, float *out, void *stream);

/* pixel2cam_torch (utils.py:356-375): depth [B][n], pix [B][3][n], ki [B][9]
 * -> cam [B][3 or 4][n] */
int mpiv_pixel2cam(const float *depth, const float *pix, const float *ki, int B, int64_t n, int homogeneous,
                   float *cam, void *stream);

/* cam2pixel_torch (utils.py:377-393): cam [B][4][n], proj [B][16] -> out [B][n][2] */
int mpiv_cam2pixel(const float *cam, const float *proj, int B, int64_t n, float *out, void *stream);

/* transform_plane_imgs_torch coordinates (utils.py:176-188): pts [M][n][3],
 * homs [M][9] -> coords [M][n][2] = (u/w/(Ht-1), v/w/(Wt-1)) */
int mpiv_plane_coords(const float *pts, int M, int64_t n, const float *homs, int Ht, int Wt, float *coords,
                      void *stream);

/* ---- frame codec ------------------------------------------------------------ */

/* preprocess_image_torch (utils.py:334-342): out = in*2 - 1, n contiguous floats */
int mpiv_preprocess(const float *in, int64_t n, float *out, void *stream);

/* deprocess_image_torch (utils.py:344-352): out = uint8(((in+1)/2)*255) with torch's
 * CPU cast semantics (truncate to int32, keep the low byte; NaN / out of int32 -> 0) */
int mpiv_deprocess_u8(const float *in, int64_t n, uint8_t *out, void *stream);

/* ---- synthetic workloads ------------------------------------------------------ */

/* Counter-based synthetic MPI (BASELINE config 5 is 36.2 GB: each GPU generates its
 * plane shard in HBM).  Writes planes [p_begin, p_end) of the MPI defined by `seed`
 * in the packed layout of mpiv_pack_planes: packed [p_end-p_begin][H+4][W+4][4] with
 * the zero border.  Texel (p, y, x, c) depends only on (seed, p, y*W+x, c) -- plane
 * indices are global, so shards generated separately equal the same planes of the
 * whole MPI bit for bit: rgb U[-1,1), alpha U[0,1), plane 0 alpha 1 (synth.hip). */
int mpiv_synth_mpi_packed(uint32_t seed, int H, int W, int p_begin, int p_end, float *packed, void *stream);

/* ---- 8-bit RGBA MPIs (the reference's test MPI is uint8 PNG; utils.py:324-331 reads
 * images as t.float() / 255) ------------------------------------------------------------ */

/* One view [H,W,P,4] uint8 (element strides strides[4] = H,W,P,C) -> packed u8 planes
 * [P][H+4][W+4] uint32 (RGBA bytes, R lowest; 4-B aligned) with a 2-texel zero border:
 * mpiv_pack_planes' layout at 4 B per texel. */
int mpiv_pack_planes_u8(const uint8_t *mpi_view, const int64_t strides[4], int H, int W, int P, uint32_t *packed,
                        void *stream);

/* mpiv_render_packed on a packed u8 MPI: out [V,H,W,3] fp32 equals mpiv_render_packed on
 * the float MPI RN(u8 / 255) bit for bit (each texel channel is converted exactly before
 * the reference's blend).  H, W >= 2. */
int mpiv_render_packed_u8(const uint32_t *packed, int H, int W, int P, const float *homs, int V, float *out,
                          void *stream);

/* mpiv_render_packed_ct on a packed u8 MPI (plane-range partial (C, T) [V,H,W,4]). */
int mpiv_render_packed_u8_ct(const uint32_t *packed, int H, int W, int P, int p_begin, int p_end, int back,
                             const float *homs, int V, float *ct, void *stream);

/* Packed u8 planes [P][H+4][W+4] -> packed float planes out [P][H+4][W+4] float4 (mpiv_pack_planes'
 * layout, 16-B aligned), every channel RN(u8 / 255) exactly: the float MPI the reference's
 * u8.float() / 255 gives (its test MPI, utils.py:324-331).  The render of many views per launch
 * converts an 8-bit MPI once with it and runs the float kernel (bit-identical frames). */
int mpiv_unpack_planes_u8(const uint32_t *packed, int H, int W, int P, float *out, void *stream);

/* Counter-based synthetic u8 MPI (mpiv_synth_mpi_packed's hash, one byte per channel =
 * the top 8 bits of its hash, plane 0 alpha 255) into the packed u8 layout. */
int mpiv_synth_mpi_packed_u8(uint32_t seed, int H, int W, int p_begin, int p_end, uint32_t *packed, void *stream);

/* ---- diagnostics ------------------------------------------------------------ */

/* Phase marker for profiles: launches an empty kernel of `tag` x 64 work-items (tag in 1..4096) on
 * the stream; tools/parse_prof.py files later dispatches under the last marker's tag. */
int mpiv_mark(int tag, void *stream);

/* Gather-rate probe (bench.py's texture-path roofline): `blocks` x 256 work-items each
 * issue iters x 8 16-B buffer loads (1 KiB per wave instruction, the render's tap shape)
 * from a 16 KiB L1/L2-resident window (window_bytes >= 16384 bytes of zeros, device, 16-B
 * aligned; smaller windows are refused); bytes moved = blocks * 256 * iters * 128.  `sink`
 * (>= 4 floats) is never written for a zero window. */
int mpiv_probe_gather(const float *window, size_t window_bytes, int iters, int blocks, float *sink, void *stream);

/* Exhaustive self-check of the render's launch-constant division (x / (H-1),
 * x / (W-1) via a precomputed reciprocal + two residual corrections) against IEEE
 * division for all 2^32 fp32 inputs and the given integer divisor; adds the number
 * of relevant mismatches to *mismatches (device counter, caller-zeroed). */
/* A/B diagnosis (libmpiv_ab.so only): the render backward fallback's ticket protocol with
 * trivial items; ctr: 4 zeroed device words (tickets, completions, violations, aborted waits),
 * marks: nphase * nvirt zeroed device ints. */
int mpiv_selftest_tickets(int blocks, int nphase, int nvirt, unsigned poll_limit, unsigned *ctr, int *marks,
                          void *stream);

int mpiv_selftest_div_const(int divisor, unsigned long long *mismatches, void *stream);

#ifdef __cplusplus
}
#endif

#endif /* MPIV_H */
