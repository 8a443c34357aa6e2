// PyTorch-ROCm custom operators over the C-ABI of libvrvq_hip.so (include/vrvq.h).
//
// TORCH_LIBRARY(vrvq, m) registers the hot-path operators as `torch.ops.vrvq.*`, with
// implementations on the CUDA (= HIP on ROCm) dispatch key. Every op:
//   - checks its tensors (device, fp32 / int dtype, contiguity) with TORCH_CHECK, so misuse is
//     a Python RuntimeError, and a C-ABI status != 0 becomes a RuntimeError with its text;
//   - allocates outputs with the torch caching allocator (at::empty) and launches on the
//     current HIP stream of the input's device (c10::hip::getCurrentHIPStream), so ops are
//     stream-ordered and capturable in a torch.cuda.CUDAGraph (no host sync, no hipMalloc);
//   - returns an empty (0-element) tensor for an output the caller did not request (the Python
//     wrappers in vrvq_amd/ops.py turn those into None).
// Fake (meta) implementations for shape propagation live in vrvq_amd/ops.py
// (torch.library.register_fake). Each op cites the reference operator it replaces.
#include <ATen/core/Tensor.h>
#include <ATen/ops/empty.h>
#include <ATen/ops/empty_like.h>
#include <ATen/ops/zeros.h>
#include <c10/core/DeviceGuard.h>
#include <c10/hip/HIPStream.h>
#include <torch/library.h>

#include "../../include/vrvq.h"

namespace {

using at::Tensor;
using c10::optional;

void* stream_of(const Tensor& t) {
  return reinterpret_cast<void*>(c10::hip::getCurrentHIPStream(t.device().index()).stream());
}

void check_rc(int rc, const char* fn) {
  TORCH_CHECK(rc == 0, fn, " failed (", rc, "): ", vrvq_status_string(rc));
}

void check_t(const Tensor& t, const char* name, at::ScalarType dt = at::kFloat) {
  TORCH_CHECK(t.is_cuda(), name, ": vrvq kernels run on the GPU only (got device ", t.device(),
              ")");
  TORCH_CHECK(t.scalar_type() == dt, name, ": expected ", dt, ", got ", t.scalar_type());
  TORCH_CHECK(t.is_contiguous(), name, ": tensor must be contiguous");
}

void check_on(const Tensor& t, const Tensor& ref, const char* name,
              at::ScalarType dt = at::kFloat) {
  check_t(t, name, dt);
  TORCH_CHECK(t.device() == ref.device(), name, ": on ", t.device(), ", expected ",
              ref.device());
}

const float* fp(const optional<Tensor>& t) {
  return t.has_value() ? t->data_ptr<float>() : nullptr;
}

void check_opt(const optional<Tensor>& t, const Tensor& ref, const char* name) {
  if (t.has_value()) check_on(*t, ref, name);
}

Tensor empty_f(at::IntArrayRef shape, const Tensor& like) {
  return at::empty(shape, like.options().dtype(at::kFloat));
}

Tensor none_like(const Tensor& like) { return at::empty({0}, like.options()); }

int64_t round_up(int64_t n, int64_t m) { return (n + m - 1) / m * m; }

// --------------------------------------------------------------------------- weights
// torch.nn.utils.weight_norm(dim=0), models/layers.py:17-22.
Tensor weight_norm(const Tensor& g, const Tensor& v) {
  check_t(g, "g");
  check_on(v, g, "v");
  c10::DeviceGuard guard(v.device());
  const int64_t rows = v.size(0), cols = v.numel() / rows;
  TORCH_CHECK(g.numel() == rows, "weight_norm: g must have one entry per row of v");
  Tensor w = at::empty_like(v);
  check_rc(vrvq_weight_norm(g.data_ptr<float>(), v.data_ptr<float>(), (int)rows, (int)cols,
                            w.data_ptr<float>(), stream_of(v)),
           "vrvq_weight_norm");
  return w;
}

// 1 / (alpha + 1e-9), models/layers.py:30.
Tensor snake_inv_alpha(const Tensor& alpha) {
  check_t(alpha, "alpha");
  c10::DeviceGuard guard(alpha.device());
  Tensor inv = at::empty_like(alpha);
  check_rc(vrvq_snake_inv_alpha(alpha.data_ptr<float>(), (int)alpha.numel(),
                                inv.data_ptr<float>(), stream_of(alpha)),
           "vrvq_snake_inv_alpha");
  return inv;
}

// F.normalize of the codebook rows + squared norms, models/quantize.py:92-99.
std::tuple<Tensor, Tensor> codebook_prep(const Tensor& cb) {
  check_t(cb, "codebook");
  c10::DeviceGuard guard(cb.device());
  const int64_t dim = cb.size(-1), rows = cb.numel() / dim;
  Tensor cbn = at::empty_like(cb);
  Tensor c2 = empty_f(cb.sizes().slice(0, cb.dim() - 1), cb);
  check_rc(vrvq_codebook_prep(cb.data_ptr<float>(), (int)rows, (int)dim, cbn.data_ptr<float>(),
                              c2.data_ptr<float>(), stream_of(cb)),
           "vrvq_codebook_prep");
  return {cbn, c2};
}

Tensor pack_conv1d_weight(const Tensor& w) {
  check_t(w, "w");
  TORCH_CHECK(w.dim() == 3, "pack_conv1d_weight: w must be (Cout, Cin, k)");
  c10::DeviceGuard guard(w.device());
  const int64_t cout = w.size(0), cin = w.size(1), k = w.size(2);
  const int64_t cout_pad = round_up(cout, 128);
  Tensor wp = empty_f({cin, k, cout_pad}, w);
  check_rc(vrvq_pack_conv1d_weight(w.data_ptr<float>(), (int)cout, (int)cin, (int)k,
                                   (int)cout_pad, wp.data_ptr<float>(), stream_of(w)),
           "vrvq_pack_conv1d_weight");
  return wp;
}

Tensor pack_convt1d_weight(const Tensor& w, int64_t stride) {
  check_t(w, "w");
  TORCH_CHECK(w.dim() == 3, "pack_convt1d_weight: w must be (Cin, Cout, k)");
  TORCH_CHECK(w.size(2) == 2 * stride,
              "conv_transpose1d: kernel_size must be 2*stride (DecoderBlock)");
  c10::DeviceGuard guard(w.device());
  const int64_t cin = w.size(0), cout = w.size(1);
  // phase rows padded to whole 128-row tiles, or 192-row tiles for strides not dividing 128
  const int64_t cout_pad = round_up(cout * stride, 128 % stride == 0 ? 128 : 192);
  Tensor wp = empty_f({cin, 2, cout_pad}, w);
  check_rc(vrvq_pack_convt1d_weight(w.data_ptr<float>(), (int)cin, (int)cout, (int)stride,
                                    (int)cout_pad, wp.data_ptr<float>(), stream_of(w)),
           "vrvq_pack_convt1d_weight");
  return wp;
}

// Pre-split bf16 weight planes for the x3 conv path (include/vrvq.h, vrvq_pack_x3_weight),
// held as int16 storage. k = taps of the packed layout (2 for a polyphase ConvTranspose1d).
Tensor pack_x3_weight(const Tensor& w_packed, int64_t k) {
  check_t(w_packed, "w_packed");
  TORCH_CHECK(w_packed.dim() == 3 && w_packed.size(1) == k,
              "pack_x3_weight: w_packed must be (Cin, k, cout_pad)");
  c10::DeviceGuard guard(w_packed.device());
  const int64_t cin = w_packed.size(0), cout_pad = w_packed.size(2);
  long long n = 0;
  check_rc(vrvq_x3_weight_size((int)cin, (int)k, (int)cout_pad, &n), "vrvq_x3_weight_size");
  Tensor w3 = at::empty({n}, w_packed.options().dtype(at::kShort));
  check_rc(vrvq_pack_x3_weight(w_packed.data_ptr<float>(), (int)cin, (int)k, (int)cout_pad,
                               reinterpret_cast<uint16_t*>(w3.data_ptr<int16_t>()),
                               stream_of(w_packed)),
           "vrvq_pack_x3_weight");
  return w3;
}

const uint16_t* x3_ptr(const optional<Tensor>& w3, const Tensor& ref, int64_t cin, int64_t k,
                       int64_t cout_pad) {
  if (!w3.has_value()) return nullptr;
  check_on(*w3, ref, "w_x3", at::kShort);
  long long n = 0;
  check_rc(vrvq_x3_weight_size((int)cin, (int)k, (int)cout_pad, &n), "vrvq_x3_weight_size");
  TORCH_CHECK(w3->numel() == n, "w_x3: expected ", n, " elements (pack_x3_weight of w_packed)");
  return reinterpret_cast<const uint16_t*>(w3->data_ptr<int16_t>());
}

// --------------------------------------------------------------------------- convs
std::tuple<Tensor, Tensor, Tensor> out_pair(const Tensor& like, at::IntArrayRef shape,
                                            const optional<Tensor>& alpha_out,
                                            const optional<Tensor>& inv_alpha_out,
                                            bool want_raw) {
  TORCH_CHECK(alpha_out.has_value() == inv_alpha_out.has_value(),
              "out_snake: alpha_out and inv_alpha_out go together");
  if (alpha_out.has_value()) {
    check_on(*alpha_out, like, "alpha_out");
    check_on(*inv_alpha_out, like, "inv_alpha_out");
    TORCH_CHECK(alpha_out->numel() == shape[1] && inv_alpha_out->numel() == shape[1],
                "out_snake: one alpha per output channel");
  }
  Tensor ys = alpha_out.has_value() ? empty_f(shape, like) : none_like(like);
  Tensor y = (want_raw || !alpha_out.has_value()) ? empty_f(shape, like) : none_like(like);
  return {y, ys, Tensor()};
}

float* opt_ptr(Tensor& t) { return t.numel() ? t.data_ptr<float>() : nullptr; }

// Snake1d -> WNConv1d (+ residual, Tanh / Sigmoid, next Snake), models/layers.py:17-41, 52-89;
// models/dac_vrvq.py:27-34, 62-74; models/importance_subnet.py:38-45.
std::tuple<Tensor, Tensor> snake_conv1d(const Tensor& x, const Tensor& w_packed, int64_t cout,
                                        int64_t stride, int64_t pad, int64_t dil,
                                        const optional<Tensor>& bias,
                                        const optional<Tensor>& alpha,
                                        const optional<Tensor>& inv_alpha,
                                        const optional<Tensor>& residual, int64_t epilogue,
                                        const optional<Tensor>& alpha_out,
                                        const optional<Tensor>& inv_alpha_out, bool want_raw,
                                        const optional<Tensor>& w_x3) {
  check_t(x, "x");
  check_on(w_packed, x, "w_packed");
  check_opt(bias, x, "bias");
  check_opt(alpha, x, "alpha");
  check_opt(inv_alpha, x, "inv_alpha");
  check_opt(residual, x, "residual");
  TORCH_CHECK(x.dim() == 3, "conv1d: x must be (B, C, T)");
  const int64_t B = x.size(0), cin = x.size(1), tin = x.size(2);
  TORCH_CHECK(w_packed.dim() == 3 && w_packed.size(0) == cin,
              "conv1d: w_packed must be (Cin, k, cout_pad) with Cin = x's channels");
  TORCH_CHECK(alpha.has_value() == inv_alpha.has_value(), "conv1d: snake needs inv_alpha");
  c10::DeviceGuard guard(x.device());
  const int64_t k = w_packed.size(1), cout_pad = w_packed.size(2);
  const int64_t tout = (tin + 2 * pad - dil * (k - 1) - 1) / stride + 1;
  TORCH_CHECK(tout > 0, "conv1d: input too short");
  if (residual.has_value())
    TORCH_CHECK(residual->sizes() == at::IntArrayRef({B, cout, tout}),
                "conv1d: residual shape must equal the output shape");
  auto [y, ys, _u] = out_pair(x, {B, cout, tout}, alpha_out, inv_alpha_out, want_raw);
  // strided conv (k = 2 stride): w_x3 holds the planes of the phase-split weight (Cin * stride
  // view channels, 2 taps; include/vrvq.h vrvq_conv1d)
  const uint16_t* w3 = stride > 1 ? x3_ptr(w_x3, x, cin * stride, 2, cout_pad)
                                  : x3_ptr(w_x3, x, cin, k, cout_pad);
  // split-K workspace of the deep-K T <= 96 layers (caching allocator: capture-safe)
  long long ws_bytes = 0;
  check_rc(vrvq_conv1d_workspace((int)B, (int)cin, (int)tin, (int)cout, (int)k, (int)stride,
                                 (int)pad, (int)dil, w3 != nullptr, &ws_bytes),
           "vrvq_conv1d_workspace");
  Tensor ws = ws_bytes > 0 ? at::empty({(ws_bytes + 3) / 4}, x.options()) : Tensor();
  check_rc(vrvq_conv1d_ws(x.data_ptr<float>(), (int)B, (int)cin, (int)tin, fp(alpha),
                          fp(inv_alpha), w_packed.data_ptr<float>(), w3, (int)cout,
                          (int)cout_pad, (int)k, (int)stride, (int)pad, (int)dil, fp(bias),
                          fp(residual), (int)epilogue, y.numel() ? y.data_ptr<float>() : nullptr,
                          (int)tout, fp(alpha_out), fp(inv_alpha_out), opt_ptr(ys),
                          ws_bytes > 0 ? ws.data_ptr() : nullptr, ws_bytes, stream_of(x)),
           "vrvq_conv1d_ws");
  return {y, ys};
}

// Snake1d -> WNConvTranspose1d (k = 2s) of DecoderBlock, models/layers.py:21-22, 92-103.
std::tuple<Tensor, Tensor> snake_conv_transpose1d(
    const Tensor& x, const Tensor& w_packed, int64_t cout, int64_t stride,
    const optional<Tensor>& bias, const optional<Tensor>& alpha,
    const optional<Tensor>& inv_alpha, const optional<Tensor>& alpha_out,
    const optional<Tensor>& inv_alpha_out, bool want_raw, int64_t pad,
    const optional<Tensor>& w_x3) {
  check_t(x, "x");
  check_on(w_packed, x, "w_packed");
  check_opt(bias, x, "bias");
  check_opt(alpha, x, "alpha");
  check_opt(inv_alpha, x, "inv_alpha");
  TORCH_CHECK(x.dim() == 3, "conv_transpose1d: x must be (B, C, T)");
  // pad -1: the DecoderBlock's ceil(stride / 2); 0: padding=False (models/dac_base.py:68-84)
  const int64_t p = pad < 0 ? (stride + 1) / 2 : pad;
  TORCH_CHECK(p < stride, "conv_transpose1d: padding must be < stride");
  TORCH_CHECK(w_packed.dim() == 3 && w_packed.size(0) == x.size(1) && w_packed.size(1) == 2,
              "conv_transpose1d: w_packed must be (Cin, 2, cout_pad)");
  TORCH_CHECK(alpha.has_value() == inv_alpha.has_value(),
              "conv_transpose1d: snake needs inv_alpha");
  c10::DeviceGuard guard(x.device());
  const int64_t B = x.size(0), cin = x.size(1), tin = x.size(2);
  const int64_t tout = (tin - 1) * stride - 2 * p + 2 * stride;
  auto [y, ys, _u] = out_pair(x, {B, cout, tout}, alpha_out, inv_alpha_out, want_raw);
  const uint16_t* w3 = x3_ptr(w_x3, x, cin, 2, w_packed.size(2));
  check_rc(vrvq_conv_transpose1d_pad(x.data_ptr<float>(), (int)B, (int)cin, (int)tin, fp(alpha),
                                     fp(inv_alpha), w_packed.data_ptr<float>(), w3, (int)cout,
                                     (int)w_packed.size(2), (int)stride, (int)p, fp(bias),
                                     opt_ptr(y), fp(alpha_out), fp(inv_alpha_out), opt_ptr(ys),
                                     stream_of(x)),
           "vrvq_conv_transpose1d_pad");
  return {y, ys};
}

// ResidualUnit in one launch, models/layers.py:52-68.
std::tuple<Tensor, Tensor> residual_unit(const Tensor& x, const Tensor& x_snk, int64_t dil,
                                         const Tensor& w7, const Tensor& b7,
                                         const Tensor& alpha2, const Tensor& inv_alpha2,
                                         const Tensor& w1, const Tensor& b1,
                                         const optional<Tensor>& alpha_out,
                                         const optional<Tensor>& inv_alpha_out, bool want_raw,
                                         const optional<Tensor>& w7_x3,
                                         const optional<Tensor>& w1_x3) {
  check_t(x, "x");
  check_on(x_snk, x, "x_snk");
  check_on(w7, x, "w7");
  check_on(b7, x, "b7");
  check_on(alpha2, x, "alpha2");
  check_on(inv_alpha2, x, "inv_alpha2");
  check_on(w1, x, "w1");
  check_on(b1, x, "b1");
  TORCH_CHECK(x.dim() == 3 && x_snk.sizes() == x.sizes(),
              "residual_unit: x_snk must have the shape of x (B, C, T)");
  c10::DeviceGuard guard(x.device());
  const int64_t B = x.size(0), C = x.size(1), T = x.size(2);
  TORCH_CHECK(w7.dim() == 3 && w7.size(0) == C && w7.size(1) == 7 && w1.dim() == 3 &&
                  w1.size(0) == C && w1.size(1) == 1 && w1.size(2) == w7.size(2),
              "residual_unit: packed weights must be (C, 7, pad) and (C, 1, pad)");
  auto [y, ys, _u] = out_pair(x, {B, C, T}, alpha_out, inv_alpha_out, want_raw);
  check_rc(vrvq_residual_unit(x.data_ptr<float>(), x_snk.data_ptr<float>(), (int)B, (int)C,
                              (int)T, (int)dil, w7.data_ptr<float>(),
                              x3_ptr(w7_x3, x, C, 7, w7.size(2)),
                              x3_ptr(w1_x3, x, C, 1, w1.size(2)), b7.data_ptr<float>(),
                              alpha2.data_ptr<float>(), inv_alpha2.data_ptr<float>(),
                              w1.data_ptr<float>(), b1.data_ptr<float>(), (int)w7.size(2),
                              opt_ptr(y), fp(alpha_out), fp(inv_alpha_out), opt_ptr(ys),
                              stream_of(x)),
           "vrvq_residual_unit");
  return {y, ys};
}

// --------------------------------------------------------------------------- RVQ
void check_rvq_weights(const Tensor& z, const Tensor& w_in_t, const Tensor& b_in,
                       const Tensor& cb, const Tensor& cbn, const Tensor& c2,
                       const Tensor& w_out, const Tensor& b_out) {
  check_on(w_in_t, z, "w_in_t");
  check_on(b_in, z, "b_in");
  check_on(cb, z, "cb");
  check_on(cbn, z, "cbn");
  check_on(c2, z, "c2");
  check_on(w_out, z, "w_out");
  check_on(b_out, z, "b_out");
  TORCH_CHECK(cb.dim() == 3 && cbn.sizes() == cb.sizes(), "rvq: cb / cbf must be (nq, N, d)");
  const int64_t nq = cb.size(0), N = cb.size(1), d = cb.size(2), D = z.size(1);
  TORCH_CHECK(c2.numel() == nq * N, "rvq: c2 must be (nq, N)");
  TORCH_CHECK(w_in_t.sizes() == at::IntArrayRef({nq, D, d}) &&
                  w_out.sizes() == at::IntArrayRef({nq, D, d}),
              "rvq: w_in_t / w_out must be (nq, D, d)");
  TORCH_CHECK(b_in.numel() == nq * d && b_out.numel() == nq * D, "rvq: bias shapes");
}

// Cross terms of the projected chain (include/vrvq.h): once per weight version.
std::tuple<Tensor, Tensor> rvq_cross_prep(const Tensor& w_in_t, const Tensor& w_out,
                                          const Tensor& b_out) {
  check_t(w_in_t, "w_in_t");
  check_on(w_out, w_in_t, "w_out");
  check_on(b_out, w_in_t, "b_out");
  TORCH_CHECK(w_in_t.dim() == 3 && w_out.sizes() == w_in_t.sizes(),
              "rvq_cross_prep: w_in_t / w_out must be (nq, D, d)");
  c10::DeviceGuard guard(w_in_t.device());
  const int64_t nq = w_in_t.size(0), D = w_in_t.size(1), d = w_in_t.size(2);
  Tensor mcol = empty_f({nq, nq, d, d}, w_in_t);
  Tensor qb = empty_f({nq, d}, w_in_t);
  check_rc(vrvq_rvq_cross_prep(w_in_t.data_ptr<float>(), w_out.data_ptr<float>(),
                               b_out.data_ptr<float>(), (int)nq, (int)D, (int)d,
                               mcol.data_ptr<float>(), qb.data_ptr<float>(), stream_of(w_in_t)),
           "vrvq_rvq_cross_prep");
  return {mcol, qb};
}

// The normalised codebooks in the chain's MFMA fragment order (include/vrvq.h, vrvq_rvq_frag).
Tensor rvq_frag(const Tensor& cbn) {
  check_t(cbn, "cbn");
  TORCH_CHECK(cbn.dim() == 3, "rvq_frag: cbn must be (nq, N, d)");
  c10::DeviceGuard guard(cbn.device());
  Tensor cbf = at::empty_like(cbn);
  check_rc(vrvq_rvq_frag(cbn.data_ptr<float>(), (int)cbn.size(0), (int)cbn.size(1),
                         (int)cbn.size(2), cbf.data_ptr<float>(), stream_of(cbn)),
           "vrvq_rvq_frag");
  return cbf;
}

// A timeout of an earlier fused RVQ launch (include/vrvq.h vrvq_rvq_pending_error): its outputs
// were poisoned (codes -1, NaN); raise here, at the next RVQ call, without synchronising.
void check_pending_rvq_error() {
  int code = 0;
  check_rc(vrvq_rvq_pending_error(&code), "vrvq_rvq_pending_error");
  TORCH_CHECK(code == 0, "vrvq: an earlier fused RVQ launch timed out in an in-kernel hand-off "
              "(code ", code, ": ", code == 1 ? "projection partials" : "stage rows",
              "); its outputs are invalid (codes -1, NaN)");
}

// VBRResidualVectorQuantize.forward quantizer loop + gating (models/quantize.py:328-443) and
// ResidualVectorQuantize.forward in eval (:136-214): all stages, z_q_is, mask, masked z_q.
// The three launches' workspace comes from the caching allocator (stream-ordered reuse).
std::tuple<Tensor, Tensor, Tensor, Tensor, Tensor, Tensor> rvq_encode(
    const Tensor& z, const Tensor& w_in_t, const Tensor& b_in, const Tensor& cb,
    const Tensor& cbf, const Tensor& c2, const Tensor& w_out, const Tensor& b_out,
    const Tensor& mcol, const Tensor& qb, const optional<Tensor>& imp, double level,
    bool want_z_q_is, bool want_mask) {
  check_pending_rvq_error();
  check_t(z, "z");
  TORCH_CHECK(z.dim() == 3, "rvq_encode: z must be (B, D, T)");
  check_rvq_weights(z, w_in_t, b_in, cb, cbf, c2, w_out, b_out);
  check_on(mcol, z, "mcol");
  check_on(qb, z, "qb");
  check_opt(imp, z, "imp");
  c10::DeviceGuard guard(z.device());
  const int64_t B = z.size(0), D = z.size(1), T = z.size(2);
  const int64_t nq = cb.size(0), N = cb.size(1), d = cb.size(2);
  TORCH_CHECK(mcol.numel() == nq * nq * d * d && qb.numel() == nq * d,
              "rvq_encode: cross terms (rvq_cross_prep) do not match nq");
  if (imp.has_value()) TORCH_CHECK(imp->numel() == B * T, "rvq_encode: imp must hold B*T values");
  Tensor codes = at::empty({B, nq, T}, z.options().dtype(at::kLong));
  Tensor latents = empty_f({B, nq * d, T}, z);
  Tensor loss_pf = empty_f({B, nq, T}, z);
  Tensor z_q_is = want_z_q_is ? empty_f({B, nq, D, T}, z) : none_like(z);
  Tensor z_q = empty_f({B, D, T}, z);
  Tensor mask = want_mask ? empty_f({B, nq, T}, z) : none_like(z);
  long long ws_bytes = 0;
  check_rc(vrvq_rvq_workspace((int)B, (int)T, (int)nq, &ws_bytes), "vrvq_rvq_workspace");
  Tensor ws = at::empty({(ws_bytes + 3) / 4}, z.options().dtype(at::kFloat));
  check_rc(vrvq_rvq_encode(z.data_ptr<float>(), (int)B, (int)D, (int)T, (int)nq, (int)N, (int)d,
                           w_in_t.data_ptr<float>(), b_in.data_ptr<float>(), cb.data_ptr<float>(),
                           cbf.data_ptr<float>(), c2.data_ptr<float>(), w_out.data_ptr<float>(),
                           b_out.data_ptr<float>(), mcol.data_ptr<float>(), qb.data_ptr<float>(),
                           fp(imp), (float)level, codes.data_ptr<int64_t>(),
                           latents.data_ptr<float>(), loss_pf.data_ptr<float>(), opt_ptr(z_q_is),
                           z_q.data_ptr<float>(), opt_ptr(mask), ws.data_ptr<float>(),
                           (long long)ws.numel() * 4, stream_of(z)),
           "vrvq_rvq_encode");
  return {codes, latents, loss_pf, z_q_is, z_q, mask};
}

// W_in planes for snake_conv1d_proj (include/vrvq.h vrvq_rvq_pack_w_in), once per weight version.
Tensor rvq_pack_w_in(const Tensor& w_in_t) {
  check_t(w_in_t, "w_in_t");
  TORCH_CHECK(w_in_t.dim() == 3, "rvq_pack_w_in: w_in_t must be (nq, D, d)");
  c10::DeviceGuard guard(w_in_t.device());
  const int64_t nq = w_in_t.size(0);
  long long n = 0;
  check_rc(vrvq_rvq_w_in_planes_size((int)nq, (int)w_in_t.size(1), (int)w_in_t.size(2), &n),
           "vrvq_rvq_w_in_planes_size");
  Tensor w3 = at::empty({n}, w_in_t.options().dtype(at::kShort));
  check_rc(vrvq_rvq_pack_w_in(w_in_t.data_ptr<float>(), (int)nq, (int)w_in_t.size(1),
                              (int)w_in_t.size(2),
                              reinterpret_cast<uint16_t*>(w3.data_ptr<int16_t>()),
                              stream_of(w_in_t)),
           "vrvq_rvq_pack_w_in");
  return w3;
}

// Snake1d -> WNConv1d (the encoder's last conv, models/dac_vrvq.py:33-34) with the in_proj of
// every RVQ stage in its epilogue (include/vrvq.h vrvq_conv1d_proj): returns the partials
// part (8, B*T, 8 nq) and, when want_z, z (B, 1024, T) as well (else an empty tensor).
std::tuple<Tensor, Tensor> snake_conv1d_proj(const Tensor& x, const Tensor& w_packed,
                                             int64_t cout, int64_t pad, int64_t dil,
                                             const optional<Tensor>& bias,
                                             const optional<Tensor>& alpha,
                                             const optional<Tensor>& inv_alpha,
                                             const optional<Tensor>& w_x3, const Tensor& w3in,
                                             int64_t nq, bool want_z) {
  check_t(x, "x");
  check_on(w_packed, x, "w_packed");
  check_opt(bias, x, "bias");
  check_opt(alpha, x, "alpha");
  check_opt(inv_alpha, x, "inv_alpha");
  check_on(w3in, x, "w3in", at::kShort);
  TORCH_CHECK(x.dim() == 3, "conv1d_proj: x must be (B, C, T)");
  TORCH_CHECK(w_packed.dim() == 3 && w_packed.size(0) == x.size(1),
              "conv1d_proj: w_packed must be (Cin, k, cout_pad) with Cin = x.shape[1]");
  TORCH_CHECK(alpha.has_value() == inv_alpha.has_value(), "conv1d_proj: snake needs inv_alpha");
  c10::DeviceGuard guard(x.device());
  const int64_t B = x.size(0), cin = x.size(1), tin = x.size(2);
  const int64_t k = w_packed.size(1), cout_pad = w_packed.size(2);
  const int64_t tout = tin + 2 * pad - dil * (k - 1);
  TORCH_CHECK(tout > 0, "conv1d_proj: input too short");
  long long n3 = 0;
  check_rc(vrvq_rvq_w_in_planes_size((int)nq, (int)cout, 8, &n3), "vrvq_rvq_w_in_planes_size");
  TORCH_CHECK(w3in.numel() == n3, "conv1d_proj: w3in must be rvq_pack_w_in(w_in_t) of nq stages");
  Tensor part = empty_f({8, B * tout, nq * 8}, x);
  Tensor z = want_z ? empty_f({B, cout, tout}, x) : none_like(x);
  const uint16_t* w3 = x3_ptr(w_x3, x, cin, k, cout_pad);
  // the split-K workspace of the shape (as snake_conv1d: the same z bits as the plain conv)
  long long ws_bytes = 0;
  check_rc(vrvq_conv1d_workspace((int)B, (int)cin, (int)tin, (int)cout, (int)k, 1, (int)pad,
                                 (int)dil, w3 != nullptr, &ws_bytes),
           "vrvq_conv1d_workspace");
  Tensor ws = ws_bytes > 0 ? at::empty({(ws_bytes + 3) / 4}, x.options()) : Tensor();
  check_rc(vrvq_conv1d_proj(x.data_ptr<float>(), (int)B, (int)cin, (int)tin, fp(alpha),
                            fp(inv_alpha), w_packed.data_ptr<float>(), w3, (int)cout,
                            (int)cout_pad, (int)k, (int)pad, (int)dil, fp(bias), opt_ptr(z),
                            (int)tout, reinterpret_cast<const uint16_t*>(w3in.data_ptr<int16_t>()),
                            (int)nq, part.data_ptr<float>(),
                            ws_bytes > 0 ? ws.data_ptr() : nullptr, ws_bytes, stream_of(x)),
           "vrvq_conv1d_proj");
  return {part, z};
}

// The quantizer from vrvq_conv1d_proj's partials (include/vrvq.h vrvq_rvq_encode_part): the
// six outputs of rvq_encode, equal to its three launches bit for bit.
std::tuple<Tensor, Tensor, Tensor, Tensor, Tensor, Tensor> rvq_encode_part(
    const Tensor& part, int64_t frames, const Tensor& b_in, const Tensor& cb, const Tensor& cbf,
    const Tensor& c2, const Tensor& w_out, const Tensor& b_out, const Tensor& mcol,
    const Tensor& qb, const optional<Tensor>& imp, double level, bool want_z_q_is,
    bool want_mask) {
  check_pending_rvq_error();
  check_t(part, "part");
  check_on(b_in, part, "b_in");
  check_on(cb, part, "cb");
  check_on(cbf, part, "cbf");
  check_on(c2, part, "c2");
  check_on(w_out, part, "w_out");
  check_on(b_out, part, "b_out");
  check_on(mcol, part, "mcol");
  check_on(qb, part, "qb");
  check_opt(imp, part, "imp");
  c10::DeviceGuard guard(part.device());
  TORCH_CHECK(cb.dim() == 3, "rvq_encode_part: cb must be (nq, N, d)");
  const int64_t nq = cb.size(0), N = cb.size(1), d = cb.size(2), T = frames;
  TORCH_CHECK(T > 0 && part.dim() == 3 && part.size(0) == 8 && part.size(2) == nq * d &&
                  part.size(1) % T == 0,
              "rvq_encode_part: part must be (8, B*T, nq*d) from conv1d_proj");
  const int64_t B = part.size(1) / T;
  TORCH_CHECK(w_out.dim() == 3 && w_out.size(0) == nq && w_out.size(2) == d,
              "rvq_encode_part: w_out must be (nq, D, d)");
  const int64_t D = w_out.size(1);
  TORCH_CHECK(b_out.numel() == nq * D && b_in.numel() == nq * d && c2.numel() == nq * N &&
                  cbf.numel() == cb.numel(),
              "rvq_encode_part: stage weights do not match cb");
  TORCH_CHECK(mcol.numel() == nq * nq * d * d && qb.numel() == nq * d,
              "rvq_encode_part: cross terms (rvq_cross_prep) do not match nq");
  if (imp.has_value()) TORCH_CHECK(imp->numel() == B * T, "rvq_encode_part: imp must hold B*T values");
  Tensor codes = at::empty({B, nq, T}, part.options().dtype(at::kLong));
  Tensor latents = empty_f({B, nq * d, T}, part);
  Tensor loss_pf = empty_f({B, nq, T}, part);
  Tensor z_q_is = want_z_q_is ? empty_f({B, nq, D, T}, part) : none_like(part);
  Tensor z_q = empty_f({B, D, T}, part);
  Tensor mask = want_mask ? empty_f({B, nq, T}, part) : none_like(part);
  long long ws_bytes = 0;
  check_rc(vrvq_rvq_workspace_part((int)B, (int)T, (int)nq, (int)N, &ws_bytes),
           "vrvq_rvq_workspace_part");
  Tensor ws = at::empty({(ws_bytes + 3) / 4}, part.options().dtype(at::kFloat));
  check_rc(vrvq_rvq_encode_part(part.data_ptr<float>(), (int)B, (int)D, (int)T, (int)nq, (int)N,
                                (int)d, b_in.data_ptr<float>(), cb.data_ptr<float>(),
                                cbf.data_ptr<float>(), c2.data_ptr<float>(),
                                w_out.data_ptr<float>(), b_out.data_ptr<float>(),
                                mcol.data_ptr<float>(), qb.data_ptr<float>(), fp(imp),
                                (float)level, codes.data_ptr<int64_t>(),
                                latents.data_ptr<float>(), loss_pf.data_ptr<float>(),
                                opt_ptr(z_q_is), z_q.data_ptr<float>(), opt_ptr(mask),
                                ws.data_ptr<float>(), (long long)ws.numel() * 4, stream_of(part)),
           "vrvq_rvq_encode_part");
  return {codes, latents, loss_pf, z_q_is, z_q, mask};
}

// Timeout code of an earlier fused RVQ launch; sync: wait for the current stream first.
int64_t rvq_check_error(const Tensor& like, bool sync) {
  int code = 0;
  if (sync && like.is_cuda()) {
    c10::DeviceGuard guard(like.device());
    check_rc(vrvq_rvq_sync_error(stream_of(like), &code), "vrvq_rvq_sync_error");
  }
  int pend = 0;
  check_rc(vrvq_rvq_pending_error(&pend), "vrvq_rvq_pending_error");
  return code ? code : pend;
}

// decode_code of every stage (models/quantize.py:81-85) for from_codes (:217-249).
// err is a 1-element int32 device tensor: 1 if a code was outside [0, N) (no host sync here;
// the Python wrapper raises IndexError like F.embedding when it is allowed to synchronise).
std::tuple<Tensor, Tensor, Tensor> rvq_gather(const Tensor& codes, const Tensor& cb) {
  check_t(codes, "codes", at::kLong);
  check_on(cb, codes, "cb");
  TORCH_CHECK(codes.dim() == 3, "rvq_gather: codes must be (B, n_codebooks, T)");
  TORCH_CHECK(cb.dim() == 3, "rvq_gather: cb must be (nq, N, d)");
  c10::DeviceGuard guard(codes.device());
  const int64_t B = codes.size(0), nq = codes.size(1), T = codes.size(2);
  TORCH_CHECK(nq <= cb.size(0), "rvq_gather: ", nq, " codebooks requested, ", cb.size(0),
              " available");
  const int64_t N = cb.size(1), d = cb.size(2);
  Tensor zst = empty_f({B, nq, T, d}, cb);
  Tensor z_p = empty_f({B, nq * d, T}, cb);
  Tensor err = at::zeros({1}, codes.options().dtype(at::kInt));
  check_rc(vrvq_rvq_gather(codes.data_ptr<int64_t>(), (int)B, (int)nq, (int)T,
                           cb.data_ptr<float>(), (int)N, (int)d, zst.data_ptr<float>(),
                           z_p.data_ptr<float>(), err.data_ptr<int>(), stream_of(codes)),
           "vrvq_rvq_gather");
  return {zst, z_p, err};
}

// decode_latents of every stage (models/quantize.py:87-103) for from_latents (:251-285).
Tensor rvq_nearest(const Tensor& latents, const Tensor& cbn, const Tensor& c2, int64_t nq) {
  check_t(latents, "latents");
  check_on(cbn, latents, "cbn");
  check_on(c2, latents, "c2");
  TORCH_CHECK(latents.dim() == 3, "from_latents: latents must be (B, N*d, T)");
  TORCH_CHECK(cbn.dim() == 3 && cbn.size(0) >= nq && c2.numel() == cbn.size(0) * cbn.size(1),
              "rvq_nearest: cbn (nq, N, d) / c2 (nq, N)");
  c10::DeviceGuard guard(latents.device());
  const int64_t B = latents.size(0), C = latents.size(1), T = latents.size(2);
  Tensor codes = at::empty({B, nq, T}, latents.options().dtype(at::kLong));
  check_rc(vrvq_rvq_nearest(latents.data_ptr<float>(), (int)B, (int)C, (int)T, (int)nq,
                            cbn.data_ptr<float>(), c2.data_ptr<float>(), (int)cbn.size(1),
                            (int)cbn.size(2), codes.data_ptr<int64_t>(), stream_of(latents)),
           "vrvq_rvq_nearest");
  return codes;
}

// out_proj of every stage from straight-through / codebook rows + (masked) sum
// (models/quantize.py:77, 217-249; scripts/inference.py:99-100).
std::tuple<Tensor, Tensor, Tensor> rvq_expand(const Tensor& zst, const Tensor& w_out,
                                              const Tensor& b_out, const optional<Tensor>& imp,
                                              double level, bool want_z_q_is, bool want_mask) {
  check_t(zst, "zst");
  check_on(w_out, zst, "w_out");
  check_on(b_out, zst, "b_out");
  check_opt(imp, zst, "imp");
  TORCH_CHECK(zst.dim() == 4, "rvq_expand: zst must be (B, nq, T, d)");
  c10::DeviceGuard guard(zst.device());
  const int64_t B = zst.size(0), nq = zst.size(1), T = zst.size(2), d = zst.size(3);
  TORCH_CHECK(w_out.dim() == 3 && w_out.size(0) >= nq && w_out.size(2) == d,
              "rvq_expand: w_out must be (>= nq, D, d)");
  const int64_t D = w_out.size(1);
  Tensor z_q_is = want_z_q_is ? empty_f({B, nq, D, T}, zst) : none_like(zst);
  Tensor z_q = empty_f({B, D, T}, zst);
  Tensor mask = want_mask ? empty_f({B, nq, T}, zst) : none_like(zst);
  check_rc(vrvq_rvq_expand(zst.data_ptr<float>(), (int)B, (int)D, (int)T, (int)nq, (int)d,
                           w_out.data_ptr<float>(), b_out.data_ptr<float>(), fp(imp),
                           (float)level, opt_ptr(z_q_is), z_q.data_ptr<float>(), opt_ptr(mask),
                           stream_of(zst)),
           "vrvq_rvq_expand");
  return {z_q_is, z_q, mask};
}

// (loss * mask).sum(1).mean(), models/quantize.py:422-423.
Tensor masked_loss(const Tensor& loss_pf, const optional<Tensor>& mask) {
  check_t(loss_pf, "loss_pf");
  check_opt(mask, loss_pf, "mask");
  TORCH_CHECK(loss_pf.dim() == 3, "masked_loss: loss_pf must be (B, nq, T)");
  c10::DeviceGuard guard(loss_pf.device());
  Tensor out = empty_f({}, loss_pf);
  check_rc(vrvq_masked_loss(loss_pf.data_ptr<float>(), fp(mask), (int)loss_pf.size(0),
                            (int)loss_pf.size(1), (int)loss_pf.size(2), out.data_ptr<float>(),
                            stream_of(loss_pf)),
           "vrvq_masked_loss");
  return out;
}

// imp_map * a * c (models/quantize.py:389, scripts/inference.py:96-97).
Tensor scale_imp(const Tensor& imp, double a, double c) {
  check_t(imp, "imp");
  c10::DeviceGuard guard(imp.device());
  Tensor s = at::empty_like(imp);
  check_rc(vrvq_scale_imp(imp.data_ptr<float>(), (int)imp.numel(), (float)a, (float)c,
                          s.data_ptr<float>(), stream_of(imp)),
           "vrvq_scale_imp");
  return s;
}

// generate_mask_hard, models/utils.py:55-61: s (B, 1, T) -> mask (B, nq, T).
Tensor imp_mask(const Tensor& s, int64_t nq) {
  check_t(s, "x");
  TORCH_CHECK(s.dim() >= 2, "generate_mask_hard: x must be (B, 1, T)");
  const int64_t B = s.size(0), T = s.size(-1);
  TORCH_CHECK(s.numel() == B * T, "generate_mask_hard: x must be (B, 1, T)");
  c10::DeviceGuard guard(s.device());
  Tensor mask = empty_f({B, nq, T}, s);
  check_rc(vrvq_mask_hard(s.data_ptr<float>(), (int)B, (int)T, (int)nq, mask.data_ptr<float>(),
                          stream_of(s)),
           "vrvq_mask_hard");
  return mask;
}

// sum_i z_q_is[:, i] * mask[:, i, None, :], scripts/inference.py:99-100.
Tensor masked_sum(const Tensor& z_q_is, const Tensor& mask) {
  check_t(z_q_is, "z_q_is");
  check_on(mask, z_q_is, "mask");
  TORCH_CHECK(z_q_is.dim() == 4, "masked_sum: z_q_is must be (B, nq, D, T)");
  const int64_t B = z_q_is.size(0), nq = z_q_is.size(1), D = z_q_is.size(2), T = z_q_is.size(3);
  TORCH_CHECK(mask.sizes() == at::IntArrayRef({B, nq, T}), "masked_sum: mask must be (B, nq, T)");
  c10::DeviceGuard guard(z_q_is.device());
  Tensor z_q = empty_f({B, D, T}, z_q_is);
  check_rc(vrvq_masked_sum(z_q_is.data_ptr<float>(), mask.data_ptr<float>(), (int)B, (int)nq,
                           (int)D, (int)T, z_q.data_ptr<float>(), stream_of(z_q_is)),
           "vrvq_masked_sum");
  return z_q;
}

// cal_bpf_from_mask, models/utils.py:64-73 (0-d device tensor, no host sync).
Tensor bpf(const Tensor& mask, const Tensor& bits) {
  check_t(mask, "mask");
  check_on(bits, mask, "bits");
  TORCH_CHECK(mask.dim() == 3, "cal_bpf_from_mask: mask must be (B, nq, T)");
  TORCH_CHECK(bits.numel() == mask.size(1), "cal_bpf_from_mask: one bit count per codebook");
  c10::DeviceGuard guard(mask.device());
  Tensor out = empty_f({}, mask);
  check_rc(vrvq_bpf(mask.data_ptr<float>(), bits.data_ptr<float>(), (int)mask.size(0),
                    (int)mask.size(1), (int)mask.size(2), out.data_ptr<float>(), stream_of(mask)),
           "vrvq_bpf");
  return out;
}

// --------------------------------------------------------------------------- code packing
// Variable-length packing. The packed length is data-dependent, so
// pack_codes takes it from the host (vrvq_amd/codes_io.py reads clip_off[B]).
std::tuple<Tensor, Tensor, Tensor> pack_counts(const Tensor& mask) {
  check_t(mask, "mask");
  TORCH_CHECK(mask.dim() == 3, "pack_counts: mask must be (B, Nq, T)");
  c10::DeviceGuard guard(mask.device());
  const int64_t B = mask.size(0), nq = mask.size(1), T = mask.size(2);
  Tensor counts = at::empty({B, T}, mask.options().dtype(at::kInt));
  Tensor tot = at::empty({B}, mask.options().dtype(at::kLong));
  Tensor off = at::empty({B + 1}, mask.options().dtype(at::kLong));
  Tensor err = at::zeros({1}, mask.options().dtype(at::kInt));
  check_rc(vrvq_pack_counts(mask.data_ptr<float>(), (int)B, (int)nq, (int)T,
                            counts.data_ptr<int>(),
                            reinterpret_cast<long long*>(tot.data_ptr<int64_t>()),
                            reinterpret_cast<long long*>(off.data_ptr<int64_t>()),
                            err.data_ptr<int>(), stream_of(mask)),
           "vrvq_pack_counts");
  return {counts, off, err};
}

std::tuple<Tensor, Tensor> pack_codes(const Tensor& codes, const Tensor& counts,
                                      const Tensor& clip_off, int64_t total, int64_t ncode) {
  check_t(codes, "codes", at::kLong);
  check_on(counts, codes, "counts", at::kInt);
  check_on(clip_off, codes, "clip_off", at::kLong);
  TORCH_CHECK(codes.dim() == 3, "pack_codes: codes must be (B, Nq, T)");
  c10::DeviceGuard guard(codes.device());
  const int64_t B = codes.size(0), nq = codes.size(1), T = codes.size(2);
  Tensor packed = at::empty({total}, codes.options().dtype(at::kShort));
  Tensor err = at::zeros({1}, codes.options().dtype(at::kInt));
  if (total > 0)
    check_rc(vrvq_pack_codes(codes.data_ptr<int64_t>(), counts.data_ptr<int>(),
                             reinterpret_cast<const long long*>(clip_off.data_ptr<int64_t>()),
                             (int)B, (int)nq, (int)T, (int)ncode,
                             reinterpret_cast<uint16_t*>(packed.data_ptr<int16_t>()),
                             err.data_ptr<int>(), stream_of(codes)),
             "vrvq_pack_codes");
  return {packed, err};
}

Tensor unpack_offsets(const Tensor& counts) {
  check_t(counts, "counts", at::kInt);
  TORCH_CHECK(counts.dim() == 2, "unpack: counts must be (B, T)");
  c10::DeviceGuard guard(counts.device());
  const int64_t B = counts.size(0), T = counts.size(1);
  Tensor tot = at::empty({B}, counts.options().dtype(at::kLong));
  Tensor off = at::empty({B + 1}, counts.options().dtype(at::kLong));
  check_rc(vrvq_unpack_offsets(counts.data_ptr<int>(), (int)B, (int)T,
                               reinterpret_cast<long long*>(tot.data_ptr<int64_t>()),
                               reinterpret_cast<long long*>(off.data_ptr<int64_t>()),
                               stream_of(counts)),
           "vrvq_unpack_offsets");
  return off;
}

std::tuple<Tensor, Tensor> unpack_codes(const Tensor& packed, const Tensor& counts,
                                        const Tensor& clip_off, int64_t n_codebooks) {
  check_t(counts, "counts", at::kInt);
  check_on(packed, counts, "packed", at::kShort);
  check_on(clip_off, counts, "clip_off", at::kLong);
  TORCH_CHECK(counts.dim() == 2 && packed.dim() == 1, "unpack: counts (B, T), packed 1-D");
  TORCH_CHECK(n_codebooks > 0 && n_codebooks <= 255, "unpack: n_codebooks in [1, 255]");
  c10::DeviceGuard guard(counts.device());
  const int64_t B = counts.size(0), T = counts.size(1);
  Tensor codes = at::empty({B, n_codebooks, T}, counts.options().dtype(at::kLong));
  Tensor mask = empty_f({B, n_codebooks, T}, counts);
  Tensor src = packed.numel() ? packed : at::zeros({1}, packed.options());
  check_rc(vrvq_unpack_codes(reinterpret_cast<const uint16_t*>(src.data_ptr<int16_t>()),
                             counts.data_ptr<int>(),
                             reinterpret_cast<const long long*>(clip_off.data_ptr<int64_t>()),
                             (int)B, (int)n_codebooks, (int)T, codes.data_ptr<int64_t>(),
                             mask.data_ptr<float>(), stream_of(counts)),
           "vrvq_unpack_codes");
  return {codes, mask};
}

// --------------------------------------------------------------------------- training step
// Backward operators of the generator (scripts/train.py:262-330), used by
// the torch.autograd.Functions of vrvq_amd/train.py.

// Strided weight gradients through the phase-split view (default) | VRVQ_WGRAD_PHASE=0: the
// strided fp32 weight-gradient kernel.
static bool phase_wgrad_enabled() {
  static const bool on = [] {
    const char* e = getenv("VRVQ_WGRAD_PHASE");
    return !(e && e[0] == '0');
  }();
  return on;
}

// torch.nn.grad.conv1d_weight of a Snake-fused conv (include/vrvq.h, vrvq_conv1d_wgrad).
Tensor conv1d_wgrad(const Tensor& a, const Tensor& x, int64_t k, int64_t stride, int64_t pad,
                    int64_t dil, const optional<Tensor>& alpha_a,
                    const optional<Tensor>& inv_alpha_a, const optional<Tensor>& alpha,
                    const optional<Tensor>& inv_alpha) {
  check_t(a, "a");
  check_on(x, a, "x");
  check_opt(alpha_a, a, "alpha_a");
  check_opt(inv_alpha_a, a, "inv_alpha_a");
  check_opt(alpha, a, "alpha");
  check_opt(inv_alpha, a, "inv_alpha");
  TORCH_CHECK(a.dim() == 3 && x.dim() == 3 && a.size(0) == x.size(0),
              "conv1d_wgrad: a (B, M, Ta) and x (B, C, Tx) with the same batch");
  TORCH_CHECK(alpha_a.has_value() == inv_alpha_a.has_value() &&
                  alpha.has_value() == inv_alpha.has_value(),
              "conv1d_wgrad: snake needs alpha and inv_alpha");
  c10::DeviceGuard guard(a.device());
  const int64_t B = a.size(0), M = a.size(1), TA = a.size(2), C = x.size(1), TX = x.size(2);
  if (alpha_a.has_value()) TORCH_CHECK(alpha_a->numel() == M, "conv1d_wgrad: alpha_a per row of a");
  if (alpha.has_value()) TORCH_CHECK(alpha->numel() == C, "conv1d_wgrad: alpha per channel of x");
  // Snake of either operand once, up front (vrvq_snake: the staging expression, so the same
  // values): the wgrad kernels would otherwise evaluate it in every row tile x chunk that
  // stages the operand (M / 64 times over for x)
  Tensor as_, xs_;
  if (stride > 1 && (stride & (stride - 1)) == 0 && k == 2 * stride && dil == 1 &&
      phase_wgrad_enabled()) {
    // strided taps j = q s + r (the strided encoder convs, the ConvTranspose layers): a stride-1
    // 2-tap product over the phase-split view xv[c s + r][m] = snake(x)[c][m s + r - pad]
    // (vrvq_phase_split, Snake applied there), on the x3 weight-gradient kernel; then
    // dW[m][c][q s + r] = dW'[m][c s + r][q]
    if (alpha_a.has_value()) {
      as_ = at::empty_like(a);
      check_rc(vrvq_snake(a.data_ptr<float>(), (int)B, (int)M, (int)TA, alpha_a->data_ptr<float>(),
                          inv_alpha_a->data_ptr<float>(), as_.data_ptr<float>(), stream_of(a)),
               "vrvq_snake");
    }
    const int64_t TV = TA + 1, CV = C * stride;
    Tensor xv = empty_f({B, CV, TV}, a);
    check_rc(vrvq_phase_split(x.data_ptr<float>(), (int)B, (int)C, (int)TX, (int)stride, (int)pad,
                              (int)TV, alpha.has_value() ? alpha->data_ptr<float>() : nullptr,
                              alpha.has_value() ? inv_alpha->data_ptr<float>() : nullptr,
                              xv.data_ptr<float>(), stream_of(a)),
             "vrvq_phase_split");
    int split = 0;
    long long bytes = 0;
    check_rc(vrvq_wgrad_plan((int)B, (int)M, (int)TA, (int)CV, 2, &split, &bytes), "vrvq_wgrad_plan");
    Tensor ws = empty_f({(bytes + 3) / 4}, a);
    Tensor outv = empty_f({M, CV, 2}, a);
    check_rc(vrvq_conv1d_wgrad(alpha_a.has_value() ? as_.data_ptr<float>() : a.data_ptr<float>(),
                               (int)B, (int)M, (int)TA, nullptr, nullptr, xv.data_ptr<float>(),
                               (int)CV, (int)TV, nullptr, nullptr, 2, 1, 0, 1, split,
                               ws.data_ptr<float>(), (long long)ws.numel() * 4,
                               outv.data_ptr<float>(), stream_of(a)),
             "vrvq_conv1d_wgrad");
    return outv.view({M, C, stride, 2}).permute({0, 1, 3, 2}).reshape({M, C, k}).contiguous();
  }
  if (alpha_a.has_value()) {
    as_ = at::empty_like(a);
    check_rc(vrvq_snake(a.data_ptr<float>(), (int)B, (int)M, (int)TA, alpha_a->data_ptr<float>(),
                        inv_alpha_a->data_ptr<float>(), as_.data_ptr<float>(), stream_of(a)),
             "vrvq_snake");
  }
  if (alpha.has_value()) {
    xs_ = at::empty_like(x);
    check_rc(vrvq_snake(x.data_ptr<float>(), (int)B, (int)C, (int)TX, alpha->data_ptr<float>(),
                        inv_alpha->data_ptr<float>(), xs_.data_ptr<float>(), stream_of(a)),
             "vrvq_snake");
  }
  int split = 0;
  long long bytes = 0;
  check_rc(vrvq_wgrad_plan((int)B, (int)M, (int)TA, (int)C, (int)k, &split, &bytes),
           "vrvq_wgrad_plan");
  Tensor ws = empty_f({(bytes + 3) / 4}, a);
  Tensor out = empty_f({M, C, k}, a);
  check_rc(vrvq_conv1d_wgrad(alpha_a.has_value() ? as_.data_ptr<float>() : a.data_ptr<float>(),
                             (int)B, (int)M, (int)TA, nullptr, nullptr,
                             alpha.has_value() ? xs_.data_ptr<float>() : x.data_ptr<float>(),
                             (int)C, (int)TX, nullptr, nullptr, (int)k, (int)stride, (int)pad,
                             (int)dil, split,
                             ws.data_ptr<float>(), (long long)ws.numel() * 4,
                             out.data_ptr<float>(), stream_of(a)),
           "vrvq_conv1d_wgrad");
  return out;
}

// Snake1d backward (models/layers.py:26-32): (dx or empty, dalpha [C]).
std::tuple<Tensor, Tensor> snake_backward(const Tensor& x, const Tensor& alpha,
                                          const Tensor& inv_alpha, const Tensor& grad,
                                          bool want_dx) {
  check_t(x, "x");
  check_on(alpha, x, "alpha");
  check_on(inv_alpha, x, "inv_alpha");
  check_on(grad, x, "grad");
  TORCH_CHECK(x.dim() == 3 && grad.sizes() == x.sizes(), "snake_backward: x, grad (B, C, T)");
  c10::DeviceGuard guard(x.device());
  const int64_t B = x.size(0), C = x.size(1), T = x.size(2);
  TORCH_CHECK(alpha.numel() == C && inv_alpha.numel() == C, "snake_backward: alpha per channel");
  long long bytes = 0;
  check_rc(vrvq_snake_backward_workspace((int)B, (int)C, (int)T, &bytes),
           "vrvq_snake_backward_workspace");
  Tensor ws = empty_f({(bytes + 3) / 4}, x);
  Tensor dx = want_dx ? at::empty_like(x) : none_like(x);
  Tensor da = empty_f({C}, x);
  check_rc(vrvq_snake_backward(x.data_ptr<float>(), alpha.data_ptr<float>(),
                               inv_alpha.data_ptr<float>(), grad.data_ptr<float>(), (int)B, (int)C,
                               (int)T, opt_ptr(dx), da.data_ptr<float>(), ws.data_ptr<float>(),
                               (long long)ws.numel() * 4, stream_of(x)),
           "vrvq_snake_backward");
  return {dx, da};
}

Tensor bias_grad(const Tensor& grad) {
  check_t(grad, "grad");
  TORCH_CHECK(grad.dim() == 3, "bias_grad: grad must be (B, C, T)");
  c10::DeviceGuard guard(grad.device());
  Tensor db = empty_f({grad.size(1)}, grad);
  long long bytes = 0;
  check_rc(vrvq_bias_grad_workspace((int)grad.size(0), (int)grad.size(1), (int)grad.size(2),
                                    &bytes),
           "vrvq_bias_grad_workspace");
  Tensor ws = empty_f({(bytes + 3) / 4}, grad);
  check_rc(vrvq_bias_grad(grad.data_ptr<float>(), (int)grad.size(0), (int)grad.size(1),
                          (int)grad.size(2), db.data_ptr<float>(), ws.data_ptr<float>(),
                          (long long)ws.numel() * 4, stream_of(grad)),
           "vrvq_bias_grad");
  return db;
}

Tensor act_backward(const Tensor& y, const Tensor& grad, int64_t epilogue) {
  check_t(y, "y");
  check_on(grad, y, "grad");
  TORCH_CHECK(grad.sizes() == y.sizes(), "act_backward: y and grad shapes differ");
  c10::DeviceGuard guard(y.device());
  Tensor out = at::empty_like(y);
  check_rc(vrvq_act_backward(y.data_ptr<float>(), grad.data_ptr<float>(), (long long)y.numel(),
                             (int)epilogue, out.data_ptr<float>(), stream_of(y)),
           "vrvq_act_backward");
  return out;
}

std::tuple<Tensor, Tensor> weight_norm_backward(const Tensor& g, const Tensor& v,
                                                const Tensor& dw) {
  check_t(g, "g");
  check_on(v, g, "v");
  check_on(dw, g, "dw");
  TORCH_CHECK(dw.sizes() == v.sizes(), "weight_norm_backward: dw must have v's shape");
  c10::DeviceGuard guard(v.device());
  const int64_t rows = v.size(0), cols = v.numel() / rows;
  TORCH_CHECK(g.numel() == rows, "weight_norm_backward: g must have one entry per row of v");
  Tensor dg = at::empty_like(g), dv = at::empty_like(v);
  check_rc(vrvq_weight_norm_backward(g.data_ptr<float>(), v.data_ptr<float>(),
                                     dw.data_ptr<float>(), (int)rows, (int)cols,
                                     dg.data_ptr<float>(), dv.data_ptr<float>(), stream_of(v)),
           "vrvq_weight_norm_backward");
  return {dg, dv};
}

// Packed adjoint of a stride-1 Conv1d weight (input gradient = conv1d of dY with it).
Tensor pack_conv1d_flip(const Tensor& w) {
  check_t(w, "w");
  TORCH_CHECK(w.dim() == 3, "pack_conv1d_flip: w must be (Cout, Cin, k)");
  c10::DeviceGuard guard(w.device());
  const int64_t cout = w.size(0), cin = w.size(1), k = w.size(2);
  const int64_t cin_pad = round_up(cin, 128);
  Tensor wp = empty_f({cout, k, cin_pad}, w);
  check_rc(vrvq_pack_conv1d_flip(w.data_ptr<float>(), (int)cout, (int)cin, (int)k, (int)cin_pad,
                                 wp.data_ptr<float>(), stream_of(w)),
           "vrvq_pack_conv1d_flip");
  return wp;
}

// Training mask (models/quantize.py:377-414).
Tensor mask_ste(const Tensor& imp, const optional<Tensor>& levels, const optional<Tensor>& dropout,
                int64_t nq, double alpha, int64_t n_imps, int64_t n_drop) {
  check_t(imp, "imp");
  if (levels.has_value()) check_on(*levels, imp, "levels");
  if (dropout.has_value()) check_on(*dropout, imp, "dropout", at::kLong);
  const int64_t B = imp.size(0), T = imp.size(-1);
  TORCH_CHECK(imp.numel() == B * T && (!levels.has_value() || levels->numel() == B),
              "mask_ste: imp (B, 1, T), levels (B)");
  if (dropout.has_value()) TORCH_CHECK(dropout->numel() == B, "mask_ste: dropout (B)");
  c10::DeviceGuard guard(imp.device());
  Tensor mask = empty_f({B, nq, T}, imp);
  check_rc(vrvq_mask_ste(imp.data_ptr<float>(),
                         levels.has_value() ? levels->data_ptr<float>() : nullptr,
                         dropout.has_value() ? dropout->data_ptr<int64_t>() : nullptr, (int)B,
                         (int)T, (int)nq, (float)alpha, (int)n_imps, (int)n_drop,
                         mask.data_ptr<float>(), stream_of(imp)),
           "vrvq_mask_ste");
  return mask;
}

Tensor mask_ste_backward(const Tensor& imp, const optional<Tensor>& levels, const Tensor& dmask,
                         double alpha, int64_t n_imps) {
  check_t(imp, "imp");
  if (levels.has_value()) check_on(*levels, imp, "levels");
  check_on(dmask, imp, "dmask");
  const int64_t B = imp.size(0), T = imp.size(-1);
  TORCH_CHECK(dmask.dim() == 3 && dmask.size(0) == B && dmask.size(2) == T,
              "mask_ste_backward: dmask (B, nq, T)");
  c10::DeviceGuard guard(imp.device());
  Tensor dimp = at::empty_like(imp);
  check_rc(vrvq_mask_ste_backward(imp.data_ptr<float>(),
                                  levels.has_value() ? levels->data_ptr<float>() : nullptr,
                                  dmask.data_ptr<float>(), (int)B, (int)T, (int)dmask.size(1),
                                  (float)alpha, (int)n_imps, dimp.data_ptr<float>(),
                                  stream_of(imp)),
           "vrvq_mask_ste_backward");
  return dimp;
}

// Training-mode quantizer forward: all stages (projection + chain) and the masked expansion
// with explicit mask values; returns the state the backward needs (zst).
std::tuple<Tensor, Tensor, Tensor, Tensor, Tensor> rvq_encode_train(
    const Tensor& z, const Tensor& w_in_t, const Tensor& b_in, const Tensor& cb,
    const Tensor& cbf, const Tensor& c2, const Tensor& w_out, const Tensor& b_out,
    const Tensor& mcol, const Tensor& qb, const Tensor& mask) {
  check_t(z, "z");
  TORCH_CHECK(z.dim() == 3, "rvq_encode_train: z must be (B, D, T)");
  check_rvq_weights(z, w_in_t, b_in, cb, cbf, c2, w_out, b_out);
  check_on(mcol, z, "mcol");
  check_on(qb, z, "qb");
  check_on(mask, z, "mask");
  c10::DeviceGuard guard(z.device());
  const int64_t B = z.size(0), D = z.size(1), T = z.size(2);
  const int64_t nq = cb.size(0), N = cb.size(1), d = cb.size(2);
  TORCH_CHECK(mask.sizes() == at::IntArrayRef({B, nq, T}), "rvq_encode_train: mask (B, nq, T)");
  TORCH_CHECK(mcol.numel() == nq * nq * d * d && qb.numel() == nq * d,
              "rvq_encode_train: cross terms (rvq_cross_prep) do not match nq");
  Tensor codes = at::empty({B, nq, T}, z.options().dtype(at::kLong));
  Tensor latents = empty_f({B, nq * d, T}, z);
  Tensor loss_pf = empty_f({B, nq, T}, z);
  Tensor zst = empty_f({B, nq, T, d}, z);
  Tensor z_q = empty_f({B, D, T}, z);
  Tensor part = empty_f({8 * B * T * nq * d}, z);
  void* st = stream_of(z);
  check_rc(vrvq_rvq_project(z.data_ptr<float>(), (int)B, (int)D, (int)T, (int)nq, (int)d,
                            w_in_t.data_ptr<float>(), part.data_ptr<float>(), st),
           "vrvq_rvq_project");
  check_rc(vrvq_rvq_chain(part.data_ptr<float>(), (int)B, (int)T, (int)nq, (int)N, (int)d,
                          b_in.data_ptr<float>(), qb.data_ptr<float>(), mcol.data_ptr<float>(),
                          cb.data_ptr<float>(), cbf.data_ptr<float>(), c2.data_ptr<float>(),
                          nullptr, 1.0f, codes.data_ptr<int64_t>(), latents.data_ptr<float>(),
                          loss_pf.data_ptr<float>(), zst.data_ptr<float>(), nullptr, st),
           "vrvq_rvq_chain");
  check_rc(vrvq_rvq_expand_masked(zst.data_ptr<float>(), (int)B, (int)D, (int)T, (int)nq, (int)d,
                                  w_out.data_ptr<float>(), b_out.data_ptr<float>(),
                                  mask.data_ptr<float>(), nullptr, z_q.data_ptr<float>(), st),
           "vrvq_rvq_expand_masked");
  return {codes, latents, loss_pf, zst, z_q};
}

std::tuple<Tensor, Tensor, Tensor, Tensor, Tensor, Tensor, Tensor> rvq_backward(
    const Tensor& dz_q, const Tensor& g_commit, const Tensor& g_codebook, const Tensor& z,
    const Tensor& zst, const Tensor& latents, const Tensor& codes, const Tensor& mask,
    const Tensor& w_in_t, const Tensor& w_out, const Tensor& b_out, const Tensor& mcol,
    const Tensor& cb) {
  check_t(dz_q, "dz_q");
  check_on(g_commit, dz_q, "g_commit");
  check_on(g_codebook, dz_q, "g_codebook");
  check_on(z, dz_q, "z");
  check_on(zst, dz_q, "zst");
  check_on(latents, dz_q, "latents");
  check_on(codes, dz_q, "codes", at::kLong);
  check_on(mask, dz_q, "mask");
  check_on(w_in_t, dz_q, "w_in_t");
  check_on(w_out, dz_q, "w_out");
  check_on(b_out, dz_q, "b_out");
  check_on(mcol, dz_q, "mcol");
  check_on(cb, dz_q, "cb");
  TORCH_CHECK(g_commit.numel() == 1 && g_codebook.numel() == 1,
              "rvq_backward: loss gradients are scalars");
  c10::DeviceGuard guard(dz_q.device());
  const int64_t B = z.size(0), D = z.size(1), T = z.size(2);
  const int64_t nq = cb.size(0), N = cb.size(1), d = cb.size(2);
  TORCH_CHECK(dz_q.sizes() == z.sizes(), "rvq_backward: dz_q must have z's shape");
  TORCH_CHECK(zst.sizes() == at::IntArrayRef({B, nq, T, d}) &&
                  latents.sizes() == at::IntArrayRef({B, nq * d, T}) &&
                  codes.sizes() == at::IntArrayRef({B, nq, T}) && mask.sizes() == codes.sizes(),
              "rvq_backward: forward state shapes");
  TORCH_CHECK(w_in_t.sizes() == at::IntArrayRef({nq, D, d}) && w_out.sizes() == w_in_t.sizes() &&
                  b_out.numel() == nq * D && mcol.numel() == nq * nq * d * d,
              "rvq_backward: weight shapes");
  long long bytes = 0;
  check_rc(vrvq_rvq_backward_workspace((int)B, (int)T, (int)nq, &bytes),
           "vrvq_rvq_backward_workspace");
  Tensor ws = empty_f({(bytes + 3) / 4}, z);
  Tensor dz = at::empty_like(z), dmask = at::empty_like(mask);
  Tensor dw_in = empty_f({nq, d, D}, z), db_in = empty_f({nq, d}, z);
  Tensor dw_out = empty_f({nq, D, d}, z), db_out = empty_f({nq, D}, z);
  Tensor dcb = at::empty_like(cb);
  check_rc(vrvq_rvq_backward(dz_q.data_ptr<float>(), g_commit.data_ptr<float>(),
                             g_codebook.data_ptr<float>(), z.data_ptr<float>(),
                             zst.data_ptr<float>(), latents.data_ptr<float>(),
                             codes.data_ptr<int64_t>(), mask.data_ptr<float>(), (int)B, (int)D,
                             (int)T, (int)nq, (int)N, (int)d, w_in_t.data_ptr<float>(),
                             w_out.data_ptr<float>(), b_out.data_ptr<float>(),
                             mcol.data_ptr<float>(), cb.data_ptr<float>(), dz.data_ptr<float>(),
                             dmask.data_ptr<float>(), dw_in.data_ptr<float>(),
                             db_in.data_ptr<float>(), dw_out.data_ptr<float>(),
                             db_out.data_ptr<float>(), dcb.data_ptr<float>(), ws.data_ptr<float>(),
                             (long long)ws.numel() * 4, stream_of(z)),
           "vrvq_rvq_backward");
  return {dz, dmask, dw_in, db_in, dw_out, db_out, dcb};
}

}  // namespace

TORCH_LIBRARY(vrvq, m) {
  m.def("weight_norm(Tensor g, Tensor v) -> Tensor");
  m.def("snake_inv_alpha(Tensor alpha) -> Tensor");
  m.def("codebook_prep(Tensor cb) -> (Tensor, Tensor)");
  m.def("pack_conv1d_weight(Tensor w) -> Tensor");
  m.def("pack_convt1d_weight(Tensor w, int stride) -> Tensor");
  m.def("pack_x3_weight(Tensor w_packed, int k) -> Tensor");
  m.def(
      "snake_conv1d(Tensor x, Tensor w_packed, int cout, int stride, int pad, int dil, "
      "Tensor? bias, Tensor? alpha, Tensor? inv_alpha, Tensor? residual, int epilogue, "
      "Tensor? alpha_out, Tensor? inv_alpha_out, bool want_raw, Tensor? w_x3=None) "
      "-> (Tensor, Tensor)");
  m.def(
      "snake_conv_transpose1d(Tensor x, Tensor w_packed, int cout, int stride, Tensor? bias, "
      "Tensor? alpha, Tensor? inv_alpha, Tensor? alpha_out, Tensor? inv_alpha_out, "
      "bool want_raw, int pad=-1, Tensor? w_x3=None) -> (Tensor, Tensor)");
  m.def(
      "residual_unit(Tensor x, Tensor x_snk, int dil, Tensor w7, Tensor b7, Tensor alpha2, "
      "Tensor inv_alpha2, Tensor w1, Tensor b1, Tensor? alpha_out, Tensor? inv_alpha_out, "
      "bool want_raw, Tensor? w7_x3=None, Tensor? w1_x3=None) -> (Tensor, Tensor)");
  m.def("rvq_cross_prep(Tensor w_in_t, Tensor w_out, Tensor b_out) -> (Tensor, Tensor)");
  m.def("rvq_frag(Tensor cbn) -> Tensor");
  m.def(
      "rvq_encode(Tensor z, Tensor w_in_t, Tensor b_in, Tensor cb, Tensor cbf, Tensor c2, "
      "Tensor w_out, Tensor b_out, Tensor mcol, Tensor qb, Tensor? imp, float level, "
      "bool want_z_q_is, bool want_mask) -> (Tensor, Tensor, Tensor, Tensor, Tensor, Tensor)");
  m.def("rvq_pack_w_in(Tensor w_in_t) -> Tensor");
  m.def(
      "snake_conv1d_proj(Tensor x, Tensor w_packed, int cout, int pad, int dil, Tensor? bias, "
      "Tensor? alpha, Tensor? inv_alpha, Tensor? w_x3, Tensor w3in, int nq, bool want_z) "
      "-> (Tensor, Tensor)");
  m.def(
      "rvq_encode_part(Tensor part, int frames, Tensor b_in, Tensor cb, Tensor cbf, Tensor c2, "
      "Tensor w_out, Tensor b_out, Tensor mcol, Tensor qb, Tensor? imp, float level, "
      "bool want_z_q_is, bool want_mask) -> (Tensor, Tensor, Tensor, Tensor, Tensor, Tensor)");
  m.def("rvq_check_error(Tensor like, bool sync) -> int");
  m.def("rvq_gather(Tensor codes, Tensor cb) -> (Tensor, Tensor, Tensor)");
  m.def("rvq_nearest(Tensor latents, Tensor cbn, Tensor c2, int nq) -> Tensor");
  m.def(
      "rvq_expand(Tensor zst, Tensor w_out, Tensor b_out, Tensor? imp, float level, "
      "bool want_z_q_is, bool want_mask) -> (Tensor, Tensor, Tensor)");
  m.def("masked_loss(Tensor loss_pf, Tensor? mask) -> Tensor");
  m.def("scale_imp(Tensor imp, float a, float c) -> Tensor");
  m.def("imp_mask(Tensor s, int nq) -> Tensor");
  m.def("masked_sum(Tensor z_q_is, Tensor mask) -> Tensor");
  m.def("bpf(Tensor mask, Tensor bits) -> Tensor");
  m.def("pack_counts(Tensor mask) -> (Tensor, Tensor, Tensor)");
  m.def(
      "pack_codes(Tensor codes, Tensor counts, Tensor clip_off, int total, int ncode) "
      "-> (Tensor, Tensor)");
  m.def("unpack_offsets(Tensor counts) -> Tensor");
  m.def(
      "unpack_codes(Tensor packed, Tensor counts, Tensor clip_off, int n_codebooks) "
      "-> (Tensor, Tensor)");
  m.def(
      "conv1d_wgrad(Tensor a, Tensor x, int k, int stride, int pad, int dil, Tensor? alpha_a, "
      "Tensor? inv_alpha_a, Tensor? alpha, Tensor? inv_alpha) -> Tensor");
  m.def(
      "snake_backward(Tensor x, Tensor alpha, Tensor inv_alpha, Tensor grad, bool want_dx) "
      "-> (Tensor, Tensor)");
  m.def("bias_grad(Tensor grad) -> Tensor");
  m.def("act_backward(Tensor y, Tensor grad, int epilogue) -> Tensor");
  m.def("weight_norm_backward(Tensor g, Tensor v, Tensor dw) -> (Tensor, Tensor)");
  m.def("pack_conv1d_flip(Tensor w) -> Tensor");
  m.def(
      "mask_ste(Tensor imp, Tensor? levels, Tensor? dropout, int nq, float alpha, int n_imps, "
      "int n_drop) -> Tensor");
  m.def(
      "mask_ste_backward(Tensor imp, Tensor? levels, Tensor dmask, float alpha, int n_imps) "
      "-> Tensor");
  m.def(
      "rvq_encode_train(Tensor z, Tensor w_in_t, Tensor b_in, Tensor cb, Tensor cbf, Tensor c2, "
      "Tensor w_out, Tensor b_out, Tensor mcol, Tensor qb, Tensor mask) "
      "-> (Tensor, Tensor, Tensor, Tensor, Tensor)");
  m.def(
      "rvq_backward(Tensor dz_q, Tensor g_commit, Tensor g_codebook, Tensor z, Tensor zst, "
      "Tensor latents, Tensor codes, Tensor mask, Tensor w_in_t, Tensor w_out, Tensor b_out, "
      "Tensor mcol, Tensor cb) -> (Tensor, Tensor, Tensor, Tensor, Tensor, Tensor, Tensor)");
}

#define VRVQ_IMPLS(m) \
  m.impl("weight_norm", &weight_norm); \
  m.impl("snake_inv_alpha", &snake_inv_alpha); \
  m.impl("codebook_prep", &codebook_prep); \
  m.impl("pack_conv1d_weight", &pack_conv1d_weight); \
  m.impl("pack_convt1d_weight", &pack_convt1d_weight); \
  m.impl("pack_x3_weight", &pack_x3_weight); \
  m.impl("snake_conv1d", &snake_conv1d); \
  m.impl("snake_conv_transpose1d", &snake_conv_transpose1d); \
  m.impl("residual_unit", &residual_unit); \
  m.impl("rvq_cross_prep", &rvq_cross_prep); \
  m.impl("rvq_frag", &rvq_frag); \
  m.impl("rvq_encode", &rvq_encode); \
  m.impl("rvq_pack_w_in", &rvq_pack_w_in); \
  m.impl("snake_conv1d_proj", &snake_conv1d_proj); \
  m.impl("rvq_encode_part", &rvq_encode_part); \
  m.impl("rvq_check_error", &rvq_check_error); \
  m.impl("rvq_gather", &rvq_gather); \
  m.impl("rvq_nearest", &rvq_nearest); \
  m.impl("rvq_expand", &rvq_expand); \
  m.impl("masked_loss", &masked_loss); \
  m.impl("scale_imp", &scale_imp); \
  m.impl("imp_mask", &imp_mask); \
  m.impl("masked_sum", &masked_sum); \
  m.impl("bpf", &bpf); \
  m.impl("pack_counts", &pack_counts); \
  m.impl("pack_codes", &pack_codes); \
  m.impl("unpack_offsets", &unpack_offsets); \
  m.impl("unpack_codes", &unpack_codes); \
  m.impl("conv1d_wgrad", &conv1d_wgrad); \
  m.impl("snake_backward", &snake_backward); \
  m.impl("bias_grad", &bias_grad); \
  m.impl("act_backward", &act_backward); \
  m.impl("weight_norm_backward", &weight_norm_backward); \
  m.impl("pack_conv1d_flip", &pack_conv1d_flip); \
  m.impl("mask_ste", &mask_ste); \
  m.impl("mask_ste_backward", &mask_ste_backward); \
  m.impl("rvq_encode_train", &rvq_encode_train); \
  m.impl("rvq_backward", &rvq_backward); \

TORCH_LIBRARY_IMPL(vrvq, CUDA, m) { VRVQ_IMPLS(m) }

// CPU tensors reach the same functions, whose first TORCH_CHECK raises "vrvq kernels run on the
// GPU only": there is no CPU fallback, and the error says so instead of a dispatcher miss.
TORCH_LIBRARY_IMPL(vrvq, CPU, m) { VRVQ_IMPLS(m) }
