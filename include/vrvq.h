/*
 * vrvq.h — C-ABI of the MI355X (gfx950) VRVQ hot path: encode -> residual VQ -> decode.
 *
 * The reference (lixinghe1999/VRVQ) has no FFI layer: its operator surface is the Python
 * module API of models/layers.py, models/quantize.py, models/utils.py and
 * models/dac_vrvq.py. Every entry point below replaces one reference operator (cited
 * file:line) and is bound from Python by ctypes in vrvq_amd/_lib.py (INTEGRATION.md shows
 * the binding a maintainer would add on the reference side).
 *
 * Conventions
 *   - All tensors are contiguous, row-major, in device (HBM) memory; fp32 unless noted.
 *   - The caller owns every buffer (inputs, outputs, workspaces); nothing is allocated here.
 *   - Every call is asynchronous on `stream` (a hipStream_t; NULL = legacy default stream)
 *     and graph-capturable (no allocation, no host sync inside).
 *   - Return value: 0 on success, otherwise a vrvq_status_t (argument errors, detected
 *     on the host before any launch) or the hipError_t of the failed launch.
 *     vrvq_status_string() turns either into text.
 */
#ifndef VRVQ_H_
#define VRVQ_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef void* vrvq_stream_t; /* hipStream_t */

enum vrvq_status_t {
  VRVQ_OK = 0,
  VRVQ_ERR_ARG = 10001,      /* null pointer / non-positive size / unsupported shape */
  VRVQ_ERR_UNSUPPORTED = 10002 /* shape outside the instantiated kernel set */
};

/* Conv epilogue selector (vrvq_conv1d.epilogue). */
enum vrvq_epilogue_t { VRVQ_EPI_NONE = 0, VRVQ_EPI_TANH = 1, VRVQ_EPI_SIGMOID = 2 };

const char* vrvq_status_string(int status);
/* Library version (major*10000 + minor*100 + patch). */
int vrvq_version(void);

/* ---------------------------------------------------------------------------------------
 * Weight preparation (once per load_state_dict; the reference recomputes weight norm on
 * every forward via the torch.nn.utils.weight_norm pre-hook).
 * ------------------------------------------------------------------------------------- */

/* w[r, :] = v[r, :] * (g[r] / ||v[r, :]||_2), r < rows, row length = cols.
 * Replaces torch.nn.utils.weight_norm(dim=0) as used by WNConv1d / WNConvTranspose1d
 * (models/layers.py:17-22). For Conv1d rows = Cout, cols = Cin*k; for ConvTranspose1d
 * rows = Cin, cols = Cout*k (weight-norm dim 0 is in_channels there). */
int vrvq_weight_norm(const float* g, const float* v, int rows, int cols, float* w,
                     vrvq_stream_t stream);

/* inv[c] = 1 / (alpha[c] + 1e-9f). Snake's reciprocal, models/layers.py:30. */
int vrvq_snake_inv_alpha(const float* alpha, int channels, float* inv, vrvq_stream_t stream);

/* y[b,c,t] = snake_c(x[b,c,t]) = x + inv_alpha[c] * sin(alpha[c] * x)^2 (Snake1d forward,
 * models/layers.py:26-32; the same per-element expression the conv kernels apply while
 * staging). The training step's weight gradients take snake(x) from here once instead of
 * re-evaluating it in every (row tile, chunk) that stages x. y may not alias x. */
int vrvq_snake(const float* x, int batch, int channels, int frames, const float* alpha,
               const float* inv_alpha, float* y, vrvq_stream_t stream);

/* Phase-split view y[b][c*stride + r][m] = snake_c(x[b][c][m*stride + r - pad]) (alpha NULL: no
 * Snake; 0 outside [0, frames)), m < out_frames, stride a power of two. Turns a stride-s
 * product over k = 2s taps (j = q s + r) into a stride-1 2-tap one: the training step's weight
 * gradients of the strided WNConv1d (models/layers.py:79-85) and WNConvTranspose1d
 * (:97-103) run on the x3 kernel over it. y may not alias x. */
int vrvq_phase_split(const float* x, int batch, int channels, int frames, int stride, int pad,
                     int out_frames, const float* alpha, const float* inv_alpha, float* y,
                     vrvq_stream_t stream);

/* Codebook normalisation for VectorQuantize.decode_latents (models/quantize.py:92-99):
 * cbn[n,:] = cb[n,:] / max(||cb[n,:]||, 1e-12); c2[n] = sum_k cbn[n,k]^2.
 * cb is [rows][dim] (rows = nq * codebook_size for a stacked RVQ). */
int vrvq_codebook_prep(const float* cb, int rows, int dim, float* cbn, float* c2,
                       vrvq_stream_t stream);

/* ---------------------------------------------------------------------------------------
 * Snake-fused 1-D convolution (implicit GEMM on v_mfma_f32_32x32x2_f32).
 *
 *   y[b,co,t] = epi( residual[b,co,t] + (bias[co] + sum_{ci,k} W[co,ci,k] *
 *                    snake_ci(x[b,ci, t*stride - pad + k*dil])) )
 *   snake_c(v) = v + inv_alpha[c] * sin(alpha[c]*v)^2     (skipped when alpha == NULL)
 *
 * Replaces Snake1d -> WNConv1d (models/layers.py:26-41, 17-18) and the ResidualUnit skip
 * (models/layers.py:63-68), EncoderBlock / Encoder / Decoder convs
 * (models/layers.py:71-89, models/dac_vrvq.py:19-80), the ImportanceSubnet convs + Sigmoid
 * (models/importance_subnet.py:38-45) and the decoder Tanh (models/dac_vrvq.py:74).
 *
 * w_packed: [Cin][k][cout_pad] (cout_pad >= Cout, multiple of 128, zero padded) as produced
 * by vrvq_pack_conv1d_weight. residual (nullable) has the output's shape.
 * tout must equal floor((tin + 2*pad - dil*(k-1) - 1)/stride) + 1.
 *
 * Producer-side Snake: when y_snake != NULL the epilogue also writes
 *   y_snake[b,co,t] = snake_co(y[b,co,t]) with alpha_out / inv_alpha_out ([Cout]),
 * i.e. the Snake1d that the NEXT layer applies to this output (models/layers.py:52-110: every
 * consumer of a conv output starts with a Snake). The consumer then runs with alpha == NULL,
 * so the activation is evaluated once per element instead of once per consumer tile. y may be
 * NULL when only the activated tensor is needed (it must not be NULL otherwise).
 * ------------------------------------------------------------------------------------- */
int vrvq_conv1d(const float* x, int batch, int cin, int tin, const float* alpha,
                const float* inv_alpha, const float* w_packed, const uint16_t* w_x3, int cout,
                int cout_pad, int k,
                int stride, int pad, int dil, const float* bias, const float* residual,
                int epilogue, float* y, int tout, const float* alpha_out,
                const float* inv_alpha_out, float* y_snake, vrvq_stream_t stream);

/* vrvq_conv1d with a caller-owned workspace (device memory, >= the bytes vrvq_conv1d_workspace
 * gives for the same shape, or NULL): the deep-K layers at tout <= 96 on the x3 path (the
 * EncoderBlock's 512 -> 1024 stride-8 conv, the ImportanceSubnet's k3 convs, the decoder's
 * first k7; models/dac_vrvq.py:32-35, 62-63, models/importance_subnet.py:38-45) then split
 * their K loop into parts whose partial sums the workspace holds, added in part order by the
 * epilogue launch. The part count depends on the layer's shape only (a clip's output does not
 * change with the batch); the sums differ from vrvq_conv1d's (unsplit) by fp32 rounding.
 * vrvq_conv1d_workspace: *bytes = 0 where no split applies (x3 = w_x3 != NULL). */
int vrvq_conv1d_workspace(int batch, int cin, int tin, int cout, int k, int stride, int pad,
                          int dil, int x3, long long* bytes);
int vrvq_conv1d_ws(const float* x, int batch, int cin, int tin, const float* alpha,
                   const float* inv_alpha, const float* w_packed, const uint16_t* w_x3, int cout,
                   int cout_pad, int k, int stride, int pad, int dil, const float* bias,
                   const float* residual, int epilogue, float* y, int tout,
                   const float* alpha_out, const float* inv_alpha_out, float* y_snake,
                   void* workspace, long long ws_bytes, vrvq_stream_t stream);

/* fp32 convolution on the bf16 matrix cores (the "x3" path, vrvq_amd/csrc/conv_x3.h): with
 * w_x3 = vrvq_pack_x3_weight(w_packed) (null: the fp32-input MFMA path) the stride-1 convs
 * (k in {1, 2, 3, 7}; also the ConvTranspose1d and the ResidualUnit's k7) split both operands
 * exactly into three bf16 terms and accumulate the six products >= 2^-16 of each fp32
 * product in fp32 — fp32 accuracy at 2.7x the MFMA ceiling. A strided conv (k = 2 stride,
 * stride a power of two: the EncoderBlock downsamplers, models/layers.py:83-88) given w_x3 runs
 * as a stride-1 2-tap conv over the phase-split view xv[c*s + r][m] = x[c][m*s + r - pad]:
 * w_x3 then holds vrvq_pack_x3_weight(cin * stride, k = 2) of the packed phase-split weight
 * W'[co][c*s + r][j] = W[co][c][j*s + r] (other strided shapes: VRVQ_ERR_UNSUPPORTED).
 * vrvq_x3_weight_size gives the buffer length in uint16 elements. */
int vrvq_x3_weight_size(int cin, int k, int cout_pad, long long* n_u16);
int vrvq_pack_x3_weight(const float* w_packed, int cin, int k, int cout_pad, uint16_t* w_x3,
                        vrvq_stream_t stream);

/* The encoder's last conv (Snake1d -> WNConv1d k3, models/dac_vrvq.py:33-34; stride 1, no
 * residual / epilogue, cout == 1024) with the in_proj of every RVQ stage in its epilogue
 * (models/quantize.py:65, VectorQuantize.in_proj applied to z for all stages at once, without
 * bias): part[s][b*tout + t][r] = sum_{c in 128 s .. 128 s + 127} W_in[r][c] z[b][c][t] for the
 * 8 channel splits s and r < 8 nq -- vrvq_rvq_project's partials bit for bit (its x3 variant),
 * computed from the conv's accumulators, so the quantizer never reads z back (vrvq_rvq_encode_part
 * takes part). w3in = vrvq_rvq_pack_w_in(w_in_t). y (nullable) also receives z [B][1024][tout]
 * as vrvq_conv1d writes it. part: [8][B*tout][8 nq] fp32, 16-byte aligned. workspace /
 * ws_bytes: as vrvq_conv1d_ws (vrvq_conv1d_workspace of the same shape; with it the conv splits
 * its K loop exactly as vrvq_conv1d_ws does, so z is the same bits either way). */
int vrvq_conv1d_proj(const float* x, int batch, int cin, int tin, const float* alpha,
                     const float* inv_alpha, const float* w_packed, const uint16_t* w_x3, int cout,
                     int cout_pad, int k, int pad, int dil, const float* bias, float* y, int tout,
                     const uint16_t* w3in, int nq, float* part, void* workspace,
                     long long ws_bytes, vrvq_stream_t stream);

/* Pack a folded Conv1d weight w[Cout][Cin][k] into [Cin][k][cout_pad]. */
int vrvq_pack_conv1d_weight(const float* w, int cout, int cin, int k, int cout_pad,
                            float* w_packed, vrvq_stream_t stream);

/* Fused ResidualUnit (models/layers.py:52-68), stride 1, k = 7 then k = 1, C channels:
 *   y = x + b1 + W1 * snake2(b7 + W7 *_dil x_snk),   x_snk = snake1(x) (given)
 * with y and / or y_snake = snake_out(y) written (as vrvq_conv1d's out_snake). The
 * intermediate snake2(...) stays in LDS. Same expressions as vrvq_conv1d(k7, out_snake =
 * snake2, no raw) followed by vrvq_conv1d(k1, residual = x) — bit-identical where both use the
 * same k7 tile height (C <= 192), else the same sums in another fp32 order. Packed by
 * vrvq_pack_conv1d_weight (same cout_pad). Supported: C in {64, 96, 128, 192, 256}, dil <= 9;
 * other C return VRVQ_ERR_UNSUPPORTED (callers use the two-launch form). w7_x3 / w1_x3
 * (nullable, vrvq_pack_x3_weight of w7_packed / w1_packed): the x3 path for the k7 GEMM and,
 * where the split hs planes fit in LDS (C = 64 / 96 / 192), the k1 GEMM. */
int vrvq_residual_unit(const float* x, const float* x_snk, int batch, int channels, int frames,
                       int dil, const float* w7_packed, const uint16_t* w7_x3,
                       const uint16_t* w1_x3, const float* b7,
                       const float* alpha2,
                       const float* inv_alpha2, const float* w1_packed, const float* b1,
                       int cout_pad, float* y, const float* alpha_out,
                       const float* inv_alpha_out, float* y_snake, vrvq_stream_t stream);

/* Snake-fused ConvTranspose1d, kernel = 2*stride, padding = stride/2 (even stride), i.e.
 * the DecoderBlock upsampler (models/layers.py:92-103): y has length tin*stride.
 * Computed as a polyphase 2-tap conv with cout*stride phase-channels:
 *   y[b,co,m*s+r-p] = bias[co] + sum_ci W[ci,co,r]*xs[ci,m] + W[ci,co,r+s]*xs[ci,m-1].
 * w_packed from vrvq_pack_convt1d_weight ([Cin][2][cout_pad]: cout*stride padded to a
 * multiple of 128, or of 192 for strides that do not divide 128). Strides 5, 7, ... return
 * VRVQ_ERR_UNSUPPORTED (a tile must hold whole output channels).
 * alpha_out / inv_alpha_out / y_snake: producer-side Snake as in vrvq_conv1d. */
int vrvq_conv_transpose1d(const float* x, int batch, int cin, int tin, const float* alpha,
                          const float* inv_alpha, const float* w_packed, int cout,
                          int cout_pad, int stride, const float* bias, float* y,
                          const float* alpha_out, const float* inv_alpha_out, float* y_snake,
                          vrvq_stream_t stream);

/* vrvq_conv_transpose1d with an explicit padding 0 <= pad < stride: y has length
 * (tin - 1)*stride - 2*pad + 2*stride. pad = 0 is the padding=False window of the chunked
 * codec (CodecMixin.padding setter, models/dac_base.py:68-84: every conv's padding -> 0). */
int vrvq_conv_transpose1d_pad(const float* x, int batch, int cin, int tin, const float* alpha,
                              const float* inv_alpha, const float* w_packed,
                              const uint16_t* w_x3, int cout,
                              int cout_pad, int stride, int pad, const float* bias, float* y,
                              const float* alpha_out, const float* inv_alpha_out,
                              float* y_snake, vrvq_stream_t stream);

/* Pack a folded ConvTranspose1d weight w[Cin][Cout][2*stride] into the polyphase layout. */
int vrvq_pack_convt1d_weight(const float* w, int cin, int cout, int stride, int cout_pad,
                             float* w_packed, vrvq_stream_t stream);

/* ---------------------------------------------------------------------------------------
 * Residual vector quantisation (VBRResidualVectorQuantize.forward, models/quantize.py:328-443;
 * per stage VectorQuantize.forward/decode_latents, models/quantize.py:42-103). Per frame (b,t)
 * and stage i:
 *   z_e   = W_in[i] r + b_in[i]                    (in_proj, WN k=1 conv D->d)
 *   e     = z_e / max(||z_e||, 1e-12)
 *   idx   = argmin_n ( (sum e^2 - 2 e.cbn[i,n]) + c2[i,n] ), lowest n on ties
 *   zq    = cb[i, idx]                             (raw codebook row)
 *   loss  = mean_k (z_e - zq)^2                    (commitment == codebook loss in forward)
 *   zst   = z_e + (zq - z_e)                       (straight-through value)
 *   r    -= W_out[i] zst + b_out[i]                (out_proj, WN k=1 conv d->D)
 * By linearity of in_proj / out_proj,
 *   z_e(i) = ((P_i + b_in[i]) - Qb_i) - sum_{j<i} M_ij zst_j,
 *   P_i = W_in[i] z,  M_ij = W_in[i] W_out[j] (8x8),  Qb_i = W_in[i] sum_{j<i} b_out[j],
 * so the sequential chain runs in the 8-dim latent space (vrvq_rvq_chain) between two
 * parallel 1024-dim passes: the projection of z for every stage (vrvq_rvq_project) and the
 * expansion of z_q_is / z_q with the reference's out_proj expression (vrvq_rvq_expand).
 *
 *   z       [B][D][T]         encoder output
 *   w_in_t  [nq][D][d]        folded in_proj weight, transposed (d fastest)
 *   b_in    [nq][d]
 *   cb      [nq][N][d]        raw codebooks; c2 [nq][N] squared norms of the normalised rows
 *   cbf     [nq][8][64][N/128][2]  normalised codebooks in the chain's MFMA fragment order
 *                             (vrvq_rvq_frag of vrvq_codebook_prep's cbn)
 *   w_out   [nq][D][d]        folded out_proj weight; b_out [nq][D]
 *   imp     [B][T] importance map, or NULL (CBR: mask = 1, models/quantize.py:397-400)
 *   level   s[b,t] = (imp[b,t] * level) * nq, mask[b,i,t] = (s - i >= 0)   (models/quantize.py:389,
 *           models/utils.py:45-61)
 * outputs:
 *   codes   [B][nq][T] int64  (torch argmax indices)
 *   latents [B][nq*d][T]      concatenated z_e
 *   loss_pf [B][nq][T]        per-frame loss
 *   z_q_is  [B][nq][D][T]     per-stage out_proj values (or NULL: not materialised)
 *   z_q     [B][D][T]         sum_i mask[b,i,t] * z_q_is[b,i,:,t], stage order
 *   mask    [B][nq][T]        (or NULL)
 * Supported: D == 1024 (latent_dim of every shipped config), d == 8, nq <= 32,
 * N % 256 == 0 and N <= 1024.
 * ------------------------------------------------------------------------------------- */

/* Once per weight version: mcol [nq][nq][d][d] with mcol[j][i] = M_ij for i > j (else 0) and
 * qb [nq][d]. */
int vrvq_rvq_cross_prep(const float* w_in_t, const float* w_out, const float* b_out, int nq,
                        int dim, int cdim, float* mcol, float* qb, vrvq_stream_t stream);

/* Once per weight version: cbf[i][w][l][t][h] = cbn[i][w*N/8 + 16t + (l&15)][4h + (l>>4)]. */
int vrvq_rvq_frag(const float* cbn, int nq, int ncode, int cdim, float* cbf,
                  vrvq_stream_t stream);

/* Projection kernel used by vrvq_rvq_project / vrvq_rvq_encode (both launch structures,
 * process-wide): 3 = one workgroup per clip x channel split on the bf16 matrix cores with both
 * operands split exactly into three bf16 terms (six products, fp32 accuracy; default); 2 = the
 * same unit on the fp32-input MFMA (an exact fmaf chain per split: the exactness fallback; also
 * VRVQ_RVQ_PROJECT=2 in the environment). 3 agrees with 2 to fp32 rounding. variant 0 queries.
 * Returns the previous variant (2 or 3), or VRVQ_ERR_ARG. */
int vrvq_rvq_project_variant(int variant);

/* Bytes of the workspace vrvq_rvq_encode needs (projection partials + straight-through rows /
 * the fused launch's stage hand-off rows, whichever is larger). */
int vrvq_rvq_workspace(int batch, int frames, int nq, long long* bytes);

/* RVQ launch structure (process-wide): 2 = fused launches (default): vrvq_rvq_encode runs ONE
 * fused launch where the shape allows it (frames <= 96; up to 32 clips per launch, more clips
 * run as consecutive launches), else its three launches; vrvq_rvq_encode_part runs rvq_pt_kernel
 * per group of resident clips. 1 = never fused: vrvq_rvq_encode's three launches,
 * vrvq_rvq_encode_part's two (chain, expansion); also VRVQ_RVQ_FUSED=0 in the environment.
 * Every structure gives the same outputs bit for bit. path 0 queries. Returns the previous path
 * (1 or 2), or VRVQ_ERR_ARG. */
int vrvq_rvq_path(int path);

/* The fused launches' in-kernel waits are bounded. A wait that runs out (a hang averted: it
 * cannot happen with the whole grid resident) records a code in the stream's sync block and in
 * a host-mapped word of the process, and the workgroup POISONS its outputs (codes -1, latents /
 * z_q / z_q_is NaN) instead of passing garbage off as results. Codes: 1 a chain part's wait for
 * the projection partials, 2 an expansion wait for a stage.
 * vrvq_rvq_sync_error: *code = the stream's word or 0, and clears it; synchronises the stream.
 * vrvq_rvq_pending_error: *code = the process word or 0 (a timeout of any launch that has
 * completed by now), and clears it; no synchronisation -- the torch ops call it at entry and
 * raise RuntimeError on a nonzero code.
 * vrvq_rvq_debug: test hook -- every later fused launch bounds its waits at spin_max polls
 * (0: the default ~0.5 s) and delays the first chain part by stall x s_sleep(127). */
int vrvq_rvq_sync_error(vrvq_stream_t stream, int* code);
int vrvq_rvq_pending_error(int* code);
int vrvq_rvq_debug(unsigned spin_max, unsigned stall);

/* Kernel timing of the fused launch (bench.py's roofline): while on (process-wide), every fused
 * launch of vrvq_rvq_encode carries a pair of HIP events in its own dispatch
 * (hipExtLaunchKernelGGL), i.e. the kernel's duration on its stream. Returns the previous
 * setting. vrvq_rvq_timing_read waits for the recorded launches and returns the mean duration
 * (ms) and their count, then forgets them. */
int vrvq_rvq_timing(int on);
int vrvq_rvq_timing_read(float* mean_ms, int* count);

/* W_in planes of vrvq_conv1d_proj's projection epilogue (once per weight version,
 * vrvq_rvq_w_in_planes_size uint16 elements): the three bf16 terms of W_in in the
 * v_mfma_f32_16x16x32_bf16 A-fragment order. */
int vrvq_rvq_w_in_planes_size(int nq, int dim, int cdim, long long* n_u16);
int vrvq_rvq_pack_w_in(const float* w_in_t, int nq, int dim, int cdim, uint16_t* w3in,
                       vrvq_stream_t stream);

/* The whole quantizer from the projection partials of vrvq_conv1d_proj (the eval encode's path):
 * ONE launch per group of resident clips (rvq_pt_kernel): chain parts (<= 16 frames of a clip)
 * sum their frames' 8 partials in split order, run the 8-dim chain and publish every stage's zst
 * rows as tagged granules; expansion workgroups (clip, 96 frames, 128 channels; one loader wave
 * polls the stage rows into LDS while seven waves write the previous stage) write z_q_is / z_q
 * under the chain. Outputs, layouts and expressions as vrvq_rvq_encode, and equal to its three
 * launches bit for bit. When a clip does not fit the resident grid (very long clips; see
 * vrvq_rvq_fused_clips) or vrvq_rvq_path(1) is set, the chain and the expansion run as two
 * stream-ordered launches over the same partials (zst rows through the workspace), with the same
 * outputs. workspace: >= vrvq_rvq_workspace_part bytes, 16-byte aligned (eager fused calls hand
 * off through the library's granule area; under stream capture the granules and the sync block
 * live in the workspace, zeroed by captured memsets). Replaces models/quantize.py:353-365,
 * 389-421 like vrvq_rvq_encode. */
int vrvq_rvq_workspace_part(int batch, int frames, int nq, int ncode, long long* bytes);
int vrvq_rvq_encode_part(const float* part, int batch, int dim, int frames, int nq, int ncode,
                         int cdim, const float* b_in, const float* cb, const float* cbf,
                         const float* c2, const float* w_out, const float* b_out,
                         const float* mcol, const float* qb, const float* imp, float level,
                         int64_t* codes, float* latents, float* loss_pf, float* z_q_is,
                         float* z_q, float* mask, void* workspace, long long workspace_bytes,
                         vrvq_stream_t stream);
/* Clips one rvq_pt_kernel launch holds resident (0: vrvq_rvq_encode_part takes its two-launch
 * form). vrvq_rvq_debug_capacity: test hook capping that number (0 forces the two launches, a
 * negative value removes the cap); returns the previous cap. */
int vrvq_rvq_fused_clips(int frames, int nq, int ncode, int* clips);
int vrvq_rvq_debug_capacity(int clips);

/* The whole quantizer, the replacement of VBRResidualVectorQuantize.forward's quantizer loop,
 * importance mask and masked sum (models/quantize.py:353-365, 389-421) and of
 * ResidualVectorQuantize.forward in eval (:136-214): one fused launch (projection units, chain
 * parts that publish every stage's zst rows, expansion workgroups that write z_q_is / z_q
 * under the chain; see vrvq_rvq_path) or three stream-ordered launches (project -> chain ->
 * expand, the steps below). The fused launch hands data between its workgroups as tagged 8-byte
 * granules (the tag carries a per-call epoch from ONE process-wide counter, so nothing needs
 * clearing between eager calls on any stream): eager calls use a library-owned granule area
 * per (device, stream), allocated with the stream's sync block on first use (hipMalloc, outside
 * any stream capture); under stream capture the granules live in the workspace, and memsets of
 * it and of the sync block are captured in front of each launch (every replay uses epoch 1).
 * workspace: >= vrvq_rvq_workspace() bytes, 16-byte aligned, caller-owned, no initialisation
 * needed. */
int vrvq_rvq_encode(const float* z, int batch, int dim, int frames, int nq, int ncode, int cdim,
                    const float* w_in_t, const float* b_in, const float* cb, const float* cbf,
                    const float* c2, const float* w_out, const float* b_out, const float* mcol,
                    const float* qb, const float* imp, float level, int64_t* codes,
                    float* latents, float* loss_pf, float* z_q_is, float* z_q, float* mask,
                    void* workspace, long long workspace_bytes, vrvq_stream_t stream);

/* Step 1: P partial sums over 8 channel splits: part [8][B*T][nq*d], part[s][b*T+t][i*d+k] =
 * sum_{c in split s} W_in[i][k][c] z[b][c][t] (in_proj without bias, all stages at once). */
int vrvq_rvq_project(const float* z, int batch, int dim, int frames, int nq, int cdim,
                     const float* w_in_t, float* part, vrvq_stream_t stream);

/* Step 2: the 8-dim chain over all nq stages (P = sum of the 8 partials in split order).
 * Outputs codes, latents (= z_e), loss_pf, zst [B][nq][T][d] (straight-through rows, the input
 * of step 3) and mask (or NULL). */
int vrvq_rvq_chain(const float* part, int batch, int frames, int nq, int ncode, int cdim,
                   const float* b_in, const float* qb, const float* mcol, const float* cb,
                   const float* cbf, const float* c2, const float* imp, float level,
                   int64_t* codes, float* latents, float* loss_pf, float* zst, float* mask,
                   vrvq_stream_t stream);

/* Step 3: HBM-streaming expansion + importance gating.
 *   z_q_is[b,i,:,t] = W_out[i] zst[b,i,t] + b_out[i]          (models/quantize.py:77)
 *   z_q[b,:,t]      = sum_i mask[b,i,t] * z_q_is[b,i,:,t]     (models/quantize.py:420-421)
 * imp == NULL: mask = 1 (CBR, and from_codes). z_q_is may be NULL (not materialised); mask, if
 * not NULL, receives the mask. Also the second half of from_codes (models/quantize.py:217-249)
 * after vrvq_rvq_gather. */
int vrvq_rvq_expand(const float* zst, int batch, int dim, int frames, int nq, int cdim,
                    const float* w_out, const float* b_out, const float* imp, float level,
                    float* z_q_is, float* z_q, float* mask, vrvq_stream_t stream);

/* Codes -> latents gather (decode_code of every stage, models/quantize.py:81-85, as used by
 * ResidualVectorQuantize.from_codes, :217-249):
 *   z_p[b, i*d + k, t] = cb[i][codes[b,i,t]][k]   (raw codebook rows, [B][nq*d][T]) or NULL
 *   zst[b][i][t][k]    = the same rows, the input layout of vrvq_rvq_expand, or NULL
 * A code outside [0, ncode) sets *err = 1 (err may be NULL) and reads row 0: the caller raises
 * IndexError as F.embedding does. */
int vrvq_rvq_gather(const int64_t* codes, int batch, int nq, int frames, const float* cb,
                    int ncode, int cdim, float* zst, float* z_p, int* err, vrvq_stream_t stream);

/* Masked loss reduction (models/quantize.py:422-423): out[0] = (loss_pf*mask).sum(1).mean().
 * One workgroup, fixed order (deterministic). */
int vrvq_masked_loss(const float* loss_pf, const float* mask, int batch, int nq, int frames,
                     float* out, vrvq_stream_t stream);

/* generate_mask_hard (models/utils.py:55-61): mask[b,n,t] = (s[b,t] - n >= 0). s is [B][T]. */
int vrvq_mask_hard(const float* s, int batch, int frames, int nq, float* mask,
                   vrvq_stream_t stream);

/* Scaled importance map: s[b,t] = (imp[b,t] * a) * c (two separate fp32 roundings, matching
 * `imp_map * level * n_codebooks` at models/quantize.py:389 with a=level, c=nq, and
 * `imp_map * (level*n_q)` at scripts/inference.py:96-97 with a=level*n_q, c=1). */
int vrvq_scale_imp(const float* imp, int n, float a, float c, float* s, vrvq_stream_t stream);

/* Masked sum over codebooks (scripts/inference.py:99-100):
 * z_q[b,:,t] = sum_i mask[b,i,t] * z_q_is[b,i,:,t]. */
int vrvq_masked_sum(const float* z_q_is, const float* mask, int batch, int nq, int dim,
                    int frames, float* z_q, vrvq_stream_t stream);

/* cal_bpf_from_mask (models/utils.py:64-73): out[0] = sum(mask*bits[n]) / (B*T). */
int vrvq_bpf(const float* mask, const float* bits, int batch, int nq, int frames, float* out,
             vrvq_stream_t stream);

/* Variable-length code packing from importance masks (the reference's
 * DACFile, models/dac_base.py:19-58, stores the full uint16 code matrix). Packed stream is
 * clip-major, frame-major, stage-minor uint16: packed[clip_off[b] + frame_off[b,t] + i] =
 * codes[b,i,t] for i < counts[b,t]; clip_off has B+1 entries (clip_off[B] = total codes).
 *   vrvq_pack_counts     mask [B][nq][T] -> counts [B*T] (int32), clip_total [B], clip_off [B+1];
 *                        *err = 1 if a mask column is not prefix-shaped (nq <= 255)
 *   vrvq_pack_codes      codes [B][nq][T] int64 -> packed (clip_off[B] uint16); *err = 2 on a
 *                        code outside [0, ncode)
 *   vrvq_unpack_offsets  counts -> clip_total, clip_off (same scan as packing)
 *   vrvq_unpack_codes    packed -> codes [B][nq][T] int64 (0 where masked) and mask or NULL */
int vrvq_pack_counts(const float* mask, int batch, int nq, int frames, int* counts,
                     long long* clip_total, long long* clip_off, int* err, vrvq_stream_t stream);
int vrvq_pack_codes(const int64_t* codes, const int* counts, const long long* clip_off, int batch,
                    int nq, int frames, int ncode, uint16_t* packed, int* err,
                    vrvq_stream_t stream);
int vrvq_unpack_offsets(const int* counts, int batch, int frames, long long* clip_total,
                        long long* clip_off, vrvq_stream_t stream);
int vrvq_unpack_codes(const uint16_t* packed, const int* counts, const long long* clip_off,
                      int batch, int nq, int frames, int64_t* codes, float* mask,
                      vrvq_stream_t stream);

/* ResidualVectorQuantize.from_latents (models/quantize.py:251-285): per stage i < nq the
 * nearest normalised codeword of the stage's own latent latents[b][8i..8i+8][t] (decode_latents,
 * :87-103; the distance expression of vrvq_rvq_chain) -> codes [B][nq][T] int64. latents has
 * nlat >= 8 nq channels; cbn [nq][ncode][8] / c2 [nq][ncode] from vrvq_codebook_prep. The
 * z_p rows and z_q follow with vrvq_rvq_gather + vrvq_rvq_expand. */
int vrvq_rvq_nearest(const float* latents, int batch, int nlat, int frames, int nq,
                     const float* cbn, const float* c2, int ncode, int cdim, int64_t* codes,
                     vrvq_stream_t stream);

/* ---------------------------------------------------------------------------------------
 * Training step (scripts/train.py:262-330): the backward operators of
 * the generator, used by the torch.autograd.Functions in vrvq_amd/train.py. Every reduction
 * runs in a fixed order (bitwise reproducible run to run).
 * ------------------------------------------------------------------------------------- */

/* Split-K plan for vrvq_conv1d_wgrad: *n_split partial sums and the workspace they need. */
int vrvq_wgrad_plan(int batch, int m, int ta, int c, int k, int* n_split,
                    long long* workspace_bytes);

/* Weight gradient of a (Snake-fused) convolution as a split-K MFMA GEMM:
 *   out[m][c][k] = sum_b sum_{t < ta} As[b][m][t] * Xs[b][c][t*stride - pad + k*dil]
 * As = snake(a) if alpha_a, Xs = snake(x) if alpha (x = 0 outside [0, tx)).
 *   WNConv1d (models/layers.py:17-18):      a = dY [B][Cout][Tout], x = layer input -> dW[Cout][Cin][k]
 *   WNConvTranspose1d (models/layers.py:21-22): a = layer input (snake on a), x = dY
 *                                           -> dW[Cin][Cout][k]
 * The autograd conv weight backward of the reference (torch.nn.grad.conv1d_weight). */
int vrvq_conv1d_wgrad(const float* a, int batch, int m, int ta, const float* alpha_a,
                      const float* inv_alpha_a, const float* x, int c, int tx, const float* alpha,
                      const float* inv_alpha, int k, int stride, int pad, int dil, int n_split,
                      float* workspace, long long workspace_bytes, float* out,
                      vrvq_stream_t stream);

/* Snake1d backward (models/layers.py:26-32): dx = g (1 + inv sin(2 a x) a) (dx may be NULL),
 * dalpha[c] = sum_{b,t} g (-inv^2 sin^2(a x) + inv sin(2 a x) x) (dalpha may be NULL). */
int vrvq_snake_backward_workspace(int batch, int channels, int frames, long long* bytes);
int vrvq_snake_backward(const float* x, const float* alpha, const float* inv_alpha,
                        const float* grad, int batch, int channels, int frames, float* dx,
                        float* dalpha, float* workspace, long long workspace_bytes,
                        vrvq_stream_t stream);

/* Conv bias gradient: db[c] = sum_{b,t} grad[b][c][t] (per-(clip, chunk) partials in the
 * workspace, summed in a fixed order). */
int vrvq_bias_grad_workspace(int batch, int channels, int frames, long long* bytes);
int vrvq_bias_grad(const float* grad, int batch, int channels, int frames, float* db,
                   float* workspace, long long workspace_bytes, vrvq_stream_t stream);

/* Tanh (models/dac_vrvq.py:74) / Sigmoid (models/importance_subnet.py:44) backward from the
 * saved output y: out = g (1 - y^2) | g y (1 - y). */
int vrvq_act_backward(const float* y, const float* grad, long long n, int epilogue, float* out,
                      vrvq_stream_t stream);

/* weight_norm backward (models/layers.py:17-22): per row, n = ||v||,
 * dg = (dw . v) / n, dv = (g / n) (dw - v (dw . v) / n^2). */
int vrvq_weight_norm_backward(const float* g, const float* v, const float* dw, int rows,
                              int cols, float* dg, float* dv, vrvq_stream_t stream);

/* Adjoint packing for the input gradient of a stride-1 Conv1d: w [cout][cin][k] ->
 * the vrvq_conv1d packed layout of W'[ci][co][k] = w[co][ci][k-1-k'] ([cout][k][cin_pad]). */
int vrvq_pack_conv1d_flip(const float* w, int cout, int cin, int k, int cin_pad,
                          float* w_packed, vrvq_stream_t stream);

/* Training-mode importance mask (models/quantize.py:377-414, models/utils.py:11-61): rows
 * b < n_imps: generate_mask_ste((imp * levels[b]) * nq, alpha) (value smooth + (hard - smooth)),
 * or, with levels == NULL, generate_mask_ste(imp, alpha) of an already scaled map;
 * the next n_drop rows n_imps + j: generate_mask_hard(dropout[j]) (the first n_drop draws, as
 * models/quantize.py:412-413 assigns dropout[:n_dropout]); the rest 1. imp [B][T], levels [B],
 * dropout [B] int64 (may be NULL when n_drop = 0), mask [B][nq][T]. */
int vrvq_mask_ste(const float* imp, const float* levels, const int64_t* dropout, int batch,
                  int frames, int nq, float alpha, int n_imps, int n_drop, float* mask,
                  vrvq_stream_t stream);
/* Its backward: dimp[b][t] = (sum_i dmask[b][i][t] logcosh'(x - i)) * nq * levels[b] for
 * b < n_imps (without the * nq * levels[b] when levels == NULL), 0 for the overwritten rows. */
int vrvq_mask_ste_backward(const float* imp, const float* levels, const float* dmask, int batch,
                           int frames, int nq, float alpha, int n_imps, float* dimp,
                           vrvq_stream_t stream);

/* vrvq_rvq_expand with explicit mask values [B][nq][T] (the training mask) instead of imp. */
int vrvq_rvq_expand_masked(const float* zst, int batch, int dim, int frames, int nq, int cdim,
                           const float* w_out, const float* b_out, const float* mask,
                           float* z_q_is, float* z_q, vrvq_stream_t stream);

/* Backward of the training-mode quantizer (models/quantize.py:42-79, 328-443): from
 * dz_q [B][D][T] and the device scalars g_commit / g_codebook (dL/d commitment_loss,
 * dL/d codebook_loss) and the forward state (z, zst [B][nq][T][d], latents [B][nq*d][T], codes,
 * mask values [B][nq][T]) computes dz [B][D][T], dmask [B][nq][T], dw_in [nq][d][D]
 * (the folded in_proj weight layout), db_in [nq][d], dw_out [nq][D][d], db_out [nq][D] and
 * dcb [nq][N][d]. D = 1024, d = 8, nq <= 32. The math (rvq_train.hip header) stays in the
 * 8-dim latent space: reverse chain with M_ji = W_in(j) W_out(i) (mcol of
 * vrvq_rvq_cross_prep), three split-K GEMMs and 8x8 fix-ups for the weight gradients. */
int vrvq_rvq_backward_workspace(int batch, int frames, int nq, long long* bytes);
int vrvq_rvq_backward(const float* dz_q, const float* g_commit, const float* g_codebook,
                      const float* z, const float* zst, const float* latents,
                      const int64_t* codes, const float* mask, int batch, int dim, int frames,
                      int nq, int ncode, int cdim, const float* w_in_t, const float* w_out,
                      const float* b_out, const float* mcol, const float* cb, float* dz,
                      float* dmask, float* dw_in, float* db_in, float* dw_out, float* db_out,
                      float* dcb, void* workspace, long long workspace_bytes,
                      vrvq_stream_t stream);

#ifdef __cplusplus
}
#endif
#endif /* VRVQ_H_ */
