// TORCH_LIBRARY(statecatcher, m): the hot-path ops of include/statecatcher.h registered with the
// PyTorch dispatcher, so they are visible to torch.compile, FakeTensor and
// torch.library.opcheck instead of being opaque ctypes calls.
//
//   CUDA (= HIP on ROCm) kernels: thin wrappers that check shapes, allocate outputs through the
//     caching allocator and call the C-ABI on the current HIP stream (no host synchronisation);
//   Meta kernels: the output shapes/dtypes only, for FakeTensor tracing;
//   autograd: registered from Python (statecatcher_amd/torch_library.py) over the *_bwd ops.
//
// Reference interfaces these replace (the Triton launches / torch calls of the hot path):
//   lucy_scan_fwd   rnn_forward_unfused_rmsnorm[(B, D)](...)      lucyrnn_triton.py:61-73, :180-244
//   lucy_scan_bwd   (absent in the reference: its Triton kernel has no backward)
//   decay_scan_fwd  fused_decay_scan[(B, D)](...)                  lucyrnn_triton.py:158-177
//   layer_norm_*    nn.LayerNorm(D) between layers                 lucyrnn_triton.py:96-97, :136-137
//   ctc_fwd/_bwd    nn.CTCLoss(blank, zero_infinity) on log_softmax  train.py:142, model.py:60-71
//   ctc_greedy_decode  decoder.py:3-30
//   mlstm_fwd/_bwd  the xLSTM encoder's mLSTM cell (fork mlstm_kernels)  model.py:214-229
//   rnnt_joint_fwd/_bwd  RNNTPredictorJoiner + log_softmax + warp_rnnt   model.py:73-145, train.py:38-42
//   gemm_tn         LinearSafe forward / input gradient GEMMs (bf16)  lucyrnn_triton.py:20-25, :107-109
//   gemm_wgrad      LinearSafe / output_proj weight gradient           lucyrnn_triton.py:20-25, :107-109
//   clip_adam_      clip_grad_norm_(params, max_norm) + optim.Adam/AdamW.step()  train.py:543-552
// There is no CPU kernel: calling an op on CPU tensors raises (no silent fallback).

#include <ATen/ATen.h>
#include <c10/core/DeviceGuard.h>
#include <c10/hip/HIPStream.h>
#include <torch/library.h>

#include <tuple>
#include <vector>

#include "statecatcher.h"

namespace {

using at::Tensor;
using c10::optional;

void sc_check(int rc, const char* what) {
  TORCH_CHECK(rc == 0, what, ": ", (rc < 0 ? "invalid argument: " : "HIP error: "),
              sc_last_error());
}

void* stream_for(const Tensor& t) {
  return (void*)c10::hip::getCurrentHIPStream(t.device().index()).stream();
}

int dtype_code(const Tensor& t) {
  switch (t.scalar_type()) {
    case at::kFloat: return SC_F32;
    case at::kBFloat16: return SC_BF16;
    case at::kHalf: return SC_F16;
    default: TORCH_CHECK(false, "statecatcher: unsupported dtype ", t.scalar_type(),
                         " (float32, bfloat16 or float16)");
  }
  return -1;
}

const void* opt_ptr(const optional<Tensor>& t) { return t && t->defined() ? t->data_ptr() : nullptr; }

// (B, T, D, gate strides bt, td, cd, cb) of [B,T,7,D] or step-blocked [B,T,D/64,7,64] gates
// (include/statecatcher.h, sc_lucy_scan_fwd)
struct GateLayout { int64_t B, T, D, bt, td, cd, cb; };

GateLayout gate_layout(const Tensor& g) {
  if (g.dim() == 4 && g.size(2) == 7 && g.stride(3) == 1)
    return {g.size(0), g.size(1), g.size(3), g.stride(0), g.stride(1), g.stride(2), 64};
  if (g.dim() == 5 && g.size(3) == 7 && g.size(4) == 64 && g.stride(4) == 1)
    return {g.size(0), g.size(1), g.size(2) * 64, g.stride(0), g.stride(1), g.stride(3), g.stride(2)};
  TORCH_CHECK(false, "statecatcher::lucy_scan: gates must be [B,T,7,D] or [B,T,D/64,7,64] with unit "
              "inner stride, got ", g.sizes(), " strides ", g.strides());
  return {};
}

// shape-only part of gate_layout (meta tensors carry strides too, but a fake [B,T,7,D] may be
// non-contiguous in the inner dim; the real kernel makes it contiguous first)
std::tuple<int64_t, int64_t, int64_t> gate_dims(const Tensor& g) {
  if (g.dim() == 4 && g.size(2) == 7) return {g.size(0), g.size(1), g.size(3)};
  if (g.dim() == 5 && g.size(3) == 7 && g.size(4) == 64) return {g.size(0), g.size(1), g.size(2) * 64};
  TORCH_CHECK(false, "statecatcher::lucy_scan: gates must be [B,T,7,D] or [B,T,D/64,7,64], got ",
              g.sizes());
  return {};
}

Tensor f32c(const Tensor& t) { return t.to(at::kFloat).contiguous(); }

// ------------------------------------------------------------------------ LucyRNN scan --------
std::tuple<Tensor, Tensor, Tensor, Tensor> lucy_scan_fwd_hip(const Tensor& gates_in, const Tensor& h0,
                                                             const Tensor& s0,
                                                             const optional<Tensor>& bias,
                                                             bool need_ckpt) {
  c10::DeviceGuard guard(gates_in.device());
  Tensor gates = gates_in;
  if (gates.dim() == 4 && gates.size(2) == 7 && gates.stride(3) != 1) gates = gates.contiguous();
  const GateLayout L = gate_layout(gates);
  TORCH_CHECK(h0.sizes() == at::IntArrayRef({L.B, L.D}) && s0.sizes() == at::IntArrayRef({L.B, L.D}),
              "statecatcher::lucy_scan_fwd: h0/s0 must be [B,D]=[", L.B, ",", L.D, "]");
  // the reference reads h0/s0 as contiguous even when handed a strided view
  Tensor h0c = f32c(h0), s0c = f32c(s0);
  optional<Tensor> bc;
  if (bias && bias->defined()) {
    TORCH_CHECK(bias->numel() == 7 * L.D, "statecatcher::lucy_scan_fwd: gate_bias must have 7*D elements");
    bc = f32c(*bias);
  }
  auto opt = gates.options();
  Tensor out = at::empty({L.B, L.T, L.D}, opt);
  Tensor s_out = at::empty({L.B, L.D}, opt.dtype(at::kFloat));
  Tensor h_out = at::empty({L.B, L.D}, opt.dtype(at::kFloat));
  Tensor ckpt = at::empty({need_ckpt ? sc_lucy_scan_ckpt_numel(L.B, L.T, L.D) : 0}, opt.dtype(at::kFloat));
  sc_check(sc_lucy_scan_fwd(gates.data_ptr(), dtype_code(gates), (const float*)opt_ptr(bc),
                            h0c.data_ptr<float>(), s0c.data_ptr<float>(), out.data_ptr(),
                            s_out.data_ptr<float>(), h_out.data_ptr<float>(), L.B, L.T, L.D, L.bt,
                            L.td, L.cd, L.cb, out.stride(0), out.stride(1),
                            need_ckpt ? ckpt.data_ptr<float>() : nullptr, stream_for(gates)),
           "statecatcher::lucy_scan_fwd");
  return {out, s_out, h_out, ckpt};
}

std::tuple<Tensor, Tensor, Tensor, Tensor> lucy_scan_fwd_meta(const Tensor& gates, const Tensor& h0,
                                                              const Tensor& s0,
                                                              const optional<Tensor>& bias,
                                                              bool need_ckpt) {
  auto [B, T, D] = gate_dims(gates);
  auto opt = gates.options();
  return {at::empty({B, T, D}, opt), at::empty({B, D}, opt.dtype(at::kFloat)),
          at::empty({B, D}, opt.dtype(at::kFloat)),
          at::empty({need_ckpt ? sc_lucy_scan_ckpt_numel(B, T, D) : 0}, opt.dtype(at::kFloat))};
}

std::tuple<Tensor, Tensor, Tensor, Tensor> lucy_scan_bwd_hip(const Tensor& gates_in, const Tensor& ckpt,
                                                             const Tensor& dout_in,
                                                             const optional<Tensor>& ds_last,
                                                             const optional<Tensor>& bias,
                                                             bool want_dbias) {
  c10::DeviceGuard guard(gates_in.device());
  // the same layouts the forward accepts: a [B,T,7,D] view strided in D is made contiguous
  Tensor gates = gates_in;
  if (gates.dim() == 4 && gates.size(2) == 7 && gates.stride(3) != 1) gates = gates.contiguous();
  const GateLayout L = gate_layout(gates);
  TORCH_CHECK(ckpt.numel() == sc_lucy_scan_ckpt_numel(L.B, L.T, L.D) && ckpt.scalar_type() == at::kFloat,
              "statecatcher::lucy_scan_bwd: ckpt is not the forward's checkpoint (run the forward "
              "with need_ckpt=True)");
  TORCH_CHECK(dout_in.sizes() == at::IntArrayRef({L.B, L.T, L.D}),
              "statecatcher::lucy_scan_bwd: dout must be [B,T,D]");
  Tensor dout = dout_in.to(gates.scalar_type());
  if (dout.stride(2) != 1) dout = dout.contiguous();
  optional<Tensor> dsl, bc;
  if (ds_last && ds_last->defined()) dsl = f32c(*ds_last);
  if (bias && bias->defined()) bc = f32c(*bias);
  Tensor dgates = at::empty(gates.sizes(), gates.options().memory_format(at::MemoryFormat::Contiguous));
  const GateLayout G = gate_layout(dgates);
  auto fo = gates.options().dtype(at::kFloat);
  Tensor dh0 = at::empty({L.B, L.D}, fo), ds0 = at::empty({L.B, L.D}, fo);
  Tensor dbias = at::empty({want_dbias ? L.B : 0, 7, L.D}, fo);
  sc_check(sc_lucy_scan_bwd(gates.data_ptr(), dtype_code(gates), (const float*)opt_ptr(bc),
                            ckpt.data_ptr<float>(), dout.data_ptr(), (const float*)opt_ptr(dsl),
                            dgates.data_ptr(), dh0.data_ptr<float>(), ds0.data_ptr<float>(),
                            want_dbias ? dbias.data_ptr<float>() : nullptr, L.B, L.T, L.D, L.bt,
                            L.td, L.cd, L.cb, dout.stride(0), dout.stride(1), G.bt, G.td, G.cd,
                            G.cb, stream_for(gates)),
           "statecatcher::lucy_scan_bwd");
  return {dgates, dh0, ds0, dbias};
}

std::tuple<Tensor, Tensor, Tensor, Tensor> lucy_scan_bwd_meta(const Tensor& gates, const Tensor& ckpt,
                                                              const Tensor& dout,
                                                              const optional<Tensor>& ds_last,
                                                              const optional<Tensor>& bias,
                                                              bool want_dbias) {
  auto [B, T, D] = gate_dims(gates);
  auto fo = gates.options().dtype(at::kFloat);
  return {at::empty(gates.sizes(), gates.options()), at::empty({B, D}, fo), at::empty({B, D}, fo),
          at::empty({want_dbias ? B : 0, 7, D}, fo)};
}

// ------------------------------------------------------------------------ decay scan ----------
void check_kv(const Tensor& kv, const Tensor& decay) {
  TORCH_CHECK(kv.dim() == 3 && kv.sizes() == decay.sizes(),
              "statecatcher::decay_scan: kv/decay must be equal [B,T,D]; got ", kv.sizes(), ", ",
              decay.sizes());
}

Tensor decay_scan_fwd_hip(const Tensor& kv_in, const Tensor& decay_in, const optional<Tensor>& init) {
  c10::DeviceGuard guard(kv_in.device());
  check_kv(kv_in, decay_in);
  Tensor kv = kv_in.contiguous(), decay = decay_in.to(kv.scalar_type()).contiguous();
  const int64_t B = kv.size(0), T = kv.size(1), D = kv.size(2);
  optional<Tensor> ic;
  if (init && init->defined()) ic = f32c(*init);
  Tensor out = at::empty_like(kv);
  sc_check(sc_decay_scan_fwd(kv.data_ptr(), decay.data_ptr(), out.data_ptr(), dtype_code(kv),
                             (const float*)opt_ptr(ic), B, T, D, kv.stride(0), kv.stride(1), 1,
                             stream_for(kv)),
           "statecatcher::decay_scan_fwd");
  return out;
}

Tensor decay_scan_fwd_meta(const Tensor& kv, const Tensor& decay, const optional<Tensor>& init) {
  check_kv(kv, decay);
  return at::empty(kv.sizes(), kv.options());
}

std::tuple<Tensor, Tensor, Tensor> decay_scan_bwd_hip(const Tensor& decay_in, const Tensor& s_all,
                                                      const Tensor& dout_in,
                                                      const optional<Tensor>& init) {
  c10::DeviceGuard guard(decay_in.device());
  check_kv(s_all, decay_in);
  Tensor decay = decay_in.to(s_all.scalar_type()).contiguous(), s = s_all.contiguous();
  Tensor dout = dout_in.to(s.scalar_type()).contiguous();
  const int64_t B = s.size(0), T = s.size(1), D = s.size(2);
  optional<Tensor> ic;
  const bool has_init = init && init->defined();
  if (has_init) ic = f32c(*init);
  Tensor dkv = at::empty_like(s), ddec = at::empty_like(s);
  Tensor dinit = at::zeros({has_init ? B : 0, D}, s.options().dtype(at::kFloat));
  sc_check(sc_decay_scan_bwd(decay.data_ptr(), s.data_ptr(), dout.data_ptr(), dkv.data_ptr(),
                             ddec.data_ptr(), dtype_code(s), (const float*)opt_ptr(ic),
                             has_init && T > 0 ? dinit.data_ptr<float>() : nullptr, B, T, D,
                             s.stride(0), s.stride(1), 1, stream_for(s)),
           "statecatcher::decay_scan_bwd");
  return {dkv, ddec, dinit};
}

std::tuple<Tensor, Tensor, Tensor> decay_scan_bwd_meta(const Tensor& decay, const Tensor& s_all,
                                                       const Tensor& dout,
                                                       const optional<Tensor>& init) {
  check_kv(s_all, decay);
  const bool has_init = init && init->defined();
  return {at::empty(s_all.sizes(), s_all.options()), at::empty(s_all.sizes(), s_all.options()),
          at::empty({has_init ? s_all.size(0) : 0, s_all.size(2)}, s_all.options().dtype(at::kFloat))};
}

// ------------------------------------------------------------------------ LayerNorm -----------
std::tuple<Tensor, Tensor, Tensor> layer_norm_fwd_hip(const Tensor& x, const Tensor& gamma,
                                                      const Tensor& beta, double eps) {
  c10::DeviceGuard guard(x.device());
  const int64_t D = x.size(-1);
  Tensor x2 = x.reshape({-1, D}).contiguous();
  const int64_t rows = x2.size(0);
  TORCH_CHECK(sc_layernorm_supported(dtype_code(x2), (int)D),
              "statecatcher::layer_norm_fwd: D=", D, " not supported for ", x2.scalar_type());
  Tensor g = f32c(gamma), b = f32c(beta);
  Tensor y = at::empty_like(x2);
  auto fo = x.options().dtype(at::kFloat);
  Tensor mean = at::empty({rows}, fo), rstd = at::empty({rows}, fo);
  sc_check(sc_layernorm_fwd(x2.data_ptr(), dtype_code(x2), g.data_ptr<float>(), b.data_ptr<float>(),
                            y.data_ptr(), mean.data_ptr<float>(), rstd.data_ptr<float>(), rows, (int)D,
                            (float)eps, stream_for(x2)),
           "statecatcher::layer_norm_fwd");
  return {y.view(x.sizes()), mean, rstd};
}

std::tuple<Tensor, Tensor, Tensor> layer_norm_fwd_meta(const Tensor& x, const Tensor& gamma,
                                                       const Tensor& beta, double eps) {
  const int64_t rows = x.numel() / std::max<int64_t>(x.size(-1), 1);
  auto fo = x.options().dtype(at::kFloat);
  return {at::empty(x.sizes(), x.options()), at::empty({rows}, fo), at::empty({rows}, fo)};
}

std::tuple<Tensor, Tensor, Tensor> layer_norm_bwd_hip(const Tensor& x, const Tensor& dy,
                                                      const Tensor& gamma, const Tensor& mean,
                                                      const Tensor& rstd) {
  c10::DeviceGuard guard(x.device());
  const int64_t D = x.size(-1);
  Tensor x2 = x.reshape({-1, D}).contiguous();
  const int64_t rows = x2.size(0);
  Tensor dy2 = dy.reshape({rows, D}).to(x2.scalar_type()).contiguous();
  Tensor g = f32c(gamma);
  Tensor dx = at::empty_like(x2);
  auto fo = x.options().dtype(at::kFloat);
  Tensor dgb = at::empty({2, D}, fo);
  Tensor ws = at::empty({sc_layernorm_bwd_workspace_numel(rows, (int)D)}, fo);
  sc_check(sc_layernorm_bwd(x2.data_ptr(), dy2.data_ptr(), dtype_code(x2), g.data_ptr<float>(),
                            mean.data_ptr<float>(), rstd.data_ptr<float>(), dx.data_ptr(),
                            dgb.data_ptr<float>(), ws.data_ptr<float>(), rows, (int)D, stream_for(x2)),
           "statecatcher::layer_norm_bwd");
  return {dx.view(x.sizes()), dgb[0], dgb[1]};
}

std::tuple<Tensor, Tensor, Tensor> layer_norm_bwd_meta(const Tensor& x, const Tensor& dy,
                                                       const Tensor& gamma, const Tensor& mean,
                                                       const Tensor& rstd) {
  auto fo = x.options().dtype(at::kFloat);
  return {at::empty(x.sizes(), x.options()), at::empty({x.size(-1)}, fo), at::empty({x.size(-1)}, fo)};
}

// ------------------------------------------------------------------------ CTC -----------------
void check_ctc(const Tensor& x, const Tensor& targets, const Tensor& in_lens, const Tensor& tgt_lens) {
  TORCH_CHECK(x.dim() == 3, "statecatcher::ctc: x must be [B,T,V], got ", x.sizes());
  TORCH_CHECK(targets.dim() == 2 && targets.size(0) == x.size(0),
              "statecatcher::ctc: targets must be padded [B, U_max] (train.py:208), got ", targets.sizes());
  TORCH_CHECK(in_lens.numel() == x.size(0) && tgt_lens.numel() == x.size(0),
              "statecatcher::ctc: in_lens/tgt_lens must have B entries");
}

int64_t ctc_ws_bytes(const Tensor& x, const Tensor& targets) {
  return (int64_t)sc_ctc_workspace_bytes((int)x.size(0), (int)std::max<int64_t>(x.size(1), 1),
                                         (int)targets.size(1));
}

std::tuple<Tensor, Tensor> ctc_fwd_hip(const Tensor& x_in, const Tensor& targets_in,
                                       const Tensor& in_lens_in, const Tensor& tgt_lens_in,
                                       int64_t blank, bool is_logits) {
  c10::DeviceGuard guard(x_in.device());
  check_ctc(x_in, targets_in, in_lens_in, tgt_lens_in);
  Tensor x = x_in.stride(2) == 1 ? x_in : x_in.contiguous();
  Tensor targets = targets_in.to(at::kLong).contiguous();
  Tensor in_lens = in_lens_in.to(at::kLong).contiguous(), tgt_lens = tgt_lens_in.to(at::kLong).contiguous();
  const int64_t B = x.size(0), T = x.size(1), V = x.size(2), umax = targets.size(1);
  const int64_t wsb = ctc_ws_bytes(x, targets);
  Tensor ws = at::empty({wsb}, x.options().dtype(at::kByte));
  if (T == 0) {   // an empty lattice: nll 0 for empty targets, +inf otherwise (ATen)
    Tensor nll = at::where(tgt_lens == 0, 0.0, std::numeric_limits<double>::infinity()).to(at::kFloat);
    return {nll, ws};
  }
  Tensor nll = at::empty({B}, x.options().dtype(at::kFloat));
  sc_check(sc_ctc_fwd(x.data_ptr(), dtype_code(x), is_logits ? 1 : 0, B, T, V, x.stride(0), x.stride(1),
                      targets.data_ptr<int64_t>(), umax ? targets.stride(0) : 0, (int)umax,
                      in_lens.data_ptr<int64_t>(), tgt_lens.data_ptr<int64_t>(), (int)blank,
                      nll.data_ptr<float>(), ws.data_ptr(), (size_t)wsb, stream_for(x)),
           "statecatcher::ctc_fwd");
  return {nll, ws};
}

std::tuple<Tensor, Tensor> ctc_fwd_meta(const Tensor& x, const Tensor& targets, const Tensor& in_lens,
                                        const Tensor& tgt_lens, int64_t blank, bool is_logits) {
  check_ctc(x, targets, in_lens, tgt_lens);
  return {at::empty({x.size(0)}, x.options().dtype(at::kFloat)),
          at::empty({ctc_ws_bytes(x, targets)}, x.options().dtype(at::kByte))};
}

Tensor ctc_bwd_hip(const Tensor& x_in, const Tensor& targets_in, const Tensor& in_lens_in,
                   const Tensor& tgt_lens_in, const Tensor& nll, const Tensor& ws, const Tensor& scale_in,
                   int64_t blank, bool is_logits) {
  c10::DeviceGuard guard(x_in.device());
  check_ctc(x_in, targets_in, in_lens_in, tgt_lens_in);
  Tensor x = x_in.stride(2) == 1 ? x_in : x_in.contiguous();
  Tensor targets = targets_in.to(at::kLong).contiguous();
  Tensor in_lens = in_lens_in.to(at::kLong).contiguous(), tgt_lens = tgt_lens_in.to(at::kLong).contiguous();
  const int64_t B = x.size(0), T = x.size(1), V = x.size(2), umax = targets.size(1);
  TORCH_CHECK(ws.numel() == ctc_ws_bytes(x, targets), "statecatcher::ctc_bwd: workspace is not ctc_fwd's");
  Tensor grad = at::empty({B, T, V}, x.options());
  if (T == 0) return grad;
  Tensor scale = f32c(scale_in.expand({B}));
  sc_check(sc_ctc_bwd(x.data_ptr(), dtype_code(x), is_logits ? 1 : 0, B, T, V, x.stride(0), x.stride(1),
                      targets.data_ptr<int64_t>(), umax ? targets.stride(0) : 0, (int)umax,
                      in_lens.data_ptr<int64_t>(), tgt_lens.data_ptr<int64_t>(), (int)blank,
                      nll.data_ptr<float>(), scale.data_ptr<float>(), grad.data_ptr(), dtype_code(grad),
                      ws.data_ptr(), (size_t)ws.numel(), stream_for(x)),
           "statecatcher::ctc_bwd");
  return grad;
}

Tensor ctc_bwd_meta(const Tensor& x, const Tensor& targets, const Tensor& in_lens, const Tensor& tgt_lens,
                    const Tensor& nll, const Tensor& ws, const Tensor& scale, int64_t blank, bool is_logits) {
  check_ctc(x, targets, in_lens, tgt_lens);
  return at::empty(x.sizes(), x.options());
}

std::tuple<Tensor, Tensor> ctc_mean_hip(const Tensor& nll, const Tensor& tgt_lens_in) {
  c10::DeviceGuard guard(nll.device());
  const int64_t B = nll.numel();
  TORCH_CHECK(tgt_lens_in.numel() == B, "statecatcher::ctc_mean: tgt_lens must have B entries");
  Tensor n = f32c(nll), tgt_lens = tgt_lens_in.to(at::kLong).contiguous();
  Tensor loss = at::empty({}, n.options()), factor = at::empty({B}, n.options());
  if (B == 0) {
    loss.fill_(std::numeric_limits<double>::quiet_NaN());   // mean over an empty batch
    return {loss, factor};
  }
  sc_check(sc_ctc_mean(n.data_ptr<float>(), tgt_lens.data_ptr<int64_t>(), (int)B, loss.data_ptr<float>(),
                       factor.data_ptr<float>(), stream_for(n)),
           "statecatcher::ctc_mean");
  return {loss, factor};
}

std::tuple<Tensor, Tensor> ctc_mean_meta(const Tensor& nll, const Tensor& tgt_lens) {
  auto fo = nll.options().dtype(at::kFloat);
  return {at::empty({}, fo), at::empty({nll.numel()}, fo)};
}

std::tuple<Tensor, Tensor> ctc_greedy_decode_hip(const Tensor& lp_in, const Tensor& lengths_in,
                                                 int64_t blank) {
  c10::DeviceGuard guard(lp_in.device());
  TORCH_CHECK(lp_in.dim() == 3, "statecatcher::ctc_greedy_decode: log_probs must be [B,T,V]");
  Tensor lp = lp_in.stride(2) == 1 ? lp_in : lp_in.contiguous();
  const int64_t B = lp.size(0), T = lp.size(1), V = lp.size(2);
  Tensor lengths = lengths_in.to(at::kLong).contiguous();
  TORCH_CHECK(lengths.numel() == B, "statecatcher::ctc_greedy_decode: lengths must have B entries");
  auto io = lp.options().dtype(at::kInt);
  Tensor tokens = at::empty({B, T}, io), counts = at::empty({B}, io);
  sc_check(sc_ctc_greedy_decode(lp.data_ptr(), dtype_code(lp), B, T, V, lp.stride(0), lp.stride(1),
                                lengths.data_ptr<int64_t>(), (int)blank, tokens.data_ptr<int32_t>(),
                                counts.data_ptr<int32_t>(), stream_for(lp)),
           "statecatcher::ctc_greedy_decode");
  return {tokens, counts};
}

std::tuple<Tensor, Tensor> ctc_greedy_decode_meta(const Tensor& lp, const Tensor& lengths, int64_t blank) {
  auto io = lp.options().dtype(at::kInt);
  return {at::empty({lp.size(0), lp.size(1)}, io), at::empty({lp.size(0)}, io)};
}

// ------------------------------------------------------------------------------ mLSTM --------
// q, k [B,NH,T,DQ], v [B,NH,T,DV] (bf16 / f16, contiguous), igate / fgate fp32 [B,NH,T]: the
// chunkwise cell of the xLSTM encoder (model.py:214-229; the fork's mlstm_kernels).
struct MlstmDims { int64_t B, NH, T, DQ, DV; };

MlstmDims check_mlstm(const Tensor& q, const Tensor& k, const Tensor& v, const Tensor& ig,
                      const Tensor& fg) {
  TORCH_CHECK(q.dim() == 4 && k.sizes() == q.sizes() && v.dim() == 4 &&
                  v.sizes().slice(0, 3) == q.sizes().slice(0, 3),
              "statecatcher::mlstm: q, k [B,NH,T,DQ] and v [B,NH,T,DV]");
  TORCH_CHECK(q.scalar_type() == k.scalar_type() && q.scalar_type() == v.scalar_type() &&
                  (q.scalar_type() == at::kBFloat16 || q.scalar_type() == at::kHalf),
              "statecatcher::mlstm: q, k, v must share a bf16 / f16 dtype");
  TORCH_CHECK(ig.sizes() == q.sizes().slice(0, 3) && fg.sizes() == ig.sizes(),
              "statecatcher::mlstm: igate / fgate must be [B,NH,T]");
  const MlstmDims d{q.size(0), q.size(1), q.size(2), q.size(3), v.size(3)};
  TORCH_CHECK(d.T % 64 == 0, "statecatcher::mlstm: T=", d.T, " must be a multiple of 64");
  TORCH_CHECK(sc_mlstm_supported(dtype_code(q), (int)d.DQ, (int)d.DV),
              "statecatcher::mlstm: head dims (", d.DQ, ", ", d.DV, ") not compiled in");
  return d;
}

std::tuple<Tensor, Tensor, Tensor, Tensor, Tensor, Tensor, Tensor> mlstm_fwd_hip(
    const Tensor& q_in, const Tensor& k_in, const Tensor& v_in, const Tensor& ig_in,
    const Tensor& fg_in, const optional<Tensor>& c0, const optional<Tensor>& n0,
    const optional<Tensor>& m0, double eps) {
  c10::DeviceGuard guard(q_in.device());
  const MlstmDims d = check_mlstm(q_in, k_in, v_in, ig_in, fg_in);
  Tensor q = q_in.contiguous(), k = k_in.contiguous(), v = v_in.contiguous();
  Tensor ig = f32c(ig_in), fg = f32c(fg_in);
  optional<Tensor> c0c, n0c, m0c;
  if (c0 && c0->defined()) c0c = f32c(*c0);
  if (n0 && n0->defined()) n0c = f32c(*n0);
  if (m0 && m0->defined()) m0c = f32c(*m0);
  const int64_t BH = d.B * d.NH, nc = d.T / 64;
  auto fo = q.options().dtype(at::kFloat);
  Tensor h = at::empty({d.B, d.NH, d.T, d.DV}, q.options());
  Tensor c_last = at::empty({d.B, d.NH, d.DQ, d.DV}, fo);
  Tensor ns = at::empty({BH, nc + 1, d.DQ}, fo), ms = at::empty({BH, nc + 1}, fo);
  Tensor cs = at::empty({BH, nc, d.DV, d.DQ}, q.options());
  Tensor mrow = at::empty({BH, d.T}, fo), den = at::empty({BH, d.T}, fo);
  sc_check(sc_mlstm_fwd(q.data_ptr(), k.data_ptr(), v.data_ptr(), dtype_code(q), ig.data_ptr<float>(),
                        fg.data_ptr<float>(), (const float*)opt_ptr(c0c), (const float*)opt_ptr(n0c),
                        (const float*)opt_ptr(m0c), (int)BH, (int)d.T, (int)d.DQ, (int)d.DV, (float)eps,
                        h.data_ptr(), cs.data_ptr(), ns.data_ptr<float>(), ms.data_ptr<float>(),
                        c_last.data_ptr<float>(), mrow.data_ptr<float>(), den.data_ptr<float>(),
                        nullptr, stream_for(q)),
           "statecatcher::mlstm_fwd");
  return {h, c_last, ns, ms, cs, mrow, den};
}

std::tuple<Tensor, Tensor, Tensor, Tensor, Tensor, Tensor, Tensor> mlstm_fwd_meta(
    const Tensor& q, const Tensor& k, const Tensor& v, const Tensor& ig, const Tensor& fg,
    const optional<Tensor>& c0, const optional<Tensor>& n0, const optional<Tensor>& m0, double eps) {
  const MlstmDims d = check_mlstm(q, k, v, ig, fg);
  const int64_t BH = d.B * d.NH, nc = d.T / 64;
  auto fo = q.options().dtype(at::kFloat);
  return {at::empty({d.B, d.NH, d.T, d.DV}, q.options()), at::empty({d.B, d.NH, d.DQ, d.DV}, fo),
          at::empty({BH, nc + 1, d.DQ}, fo), at::empty({BH, nc + 1}, fo),
          at::empty({BH, nc, d.DV, d.DQ}, q.options()), at::empty({BH, d.T}, fo),
          at::empty({BH, d.T}, fo)};
}

std::tuple<Tensor, Tensor, Tensor, Tensor, Tensor, Tensor, Tensor> mlstm_bwd_hip(
    const Tensor& q_in, const Tensor& k_in, const Tensor& v_in, const Tensor& ig_in,
    const Tensor& fg_in, const Tensor& h, const Tensor& dh_in, const optional<Tensor>& dcT,
    const optional<Tensor>& dnT, const Tensor& cs, const Tensor& ns, const Tensor& ms,
    const Tensor& mrow, const Tensor& den, double eps) {
  c10::DeviceGuard guard(q_in.device());
  const MlstmDims d = check_mlstm(q_in, k_in, v_in, ig_in, fg_in);
  Tensor q = q_in.contiguous(), k = k_in.contiguous(), v = v_in.contiguous();
  Tensor ig = f32c(ig_in), fg = f32c(fg_in);
  Tensor dh = dh_in.to(q.scalar_type()).contiguous(), hc = h.contiguous();
  TORCH_CHECK(dh.sizes() == hc.sizes() && hc.sizes() == v.sizes(),
              "statecatcher::mlstm_bwd: h / dh must be [B,NH,T,DV]");
  const int64_t BH = d.B * d.NH, nc = d.T / 64;
  TORCH_CHECK(cs.numel() == BH * nc * d.DQ * d.DV && cs.scalar_type() == q.scalar_type() &&
                  cs.is_contiguous() && cs.device() == q.device(),
              "statecatcher::mlstm_bwd: c_states is not mlstm_fwd's");
  // the other state images go to the kernel as raw pointers: shape, dtype, layout and device
  // exactly as mlstm_fwd returns them
  auto f32_state = [&](const Tensor& t, at::IntArrayRef shape, const char* name) {
    TORCH_CHECK(t.sizes() == shape && t.scalar_type() == at::kFloat && t.is_contiguous() &&
                    t.device() == q.device(),
                "statecatcher::mlstm_bwd: ", name, " must be contiguous fp32 ", shape,
                " on the device of q (mlstm_fwd's output), got ", t.sizes(), " ", t.scalar_type());
  };
  f32_state(ns, {BH, nc + 1, d.DQ}, "n_states");
  f32_state(ms, {BH, nc + 1}, "m_states");
  f32_state(mrow, {BH, d.T}, "m_rows");
  f32_state(den, {BH, d.T}, "den_rows");
  optional<Tensor> dcc, dnc;
  if (dcT && dcT->defined()) dcc = f32c(*dcT);
  if (dnT && dnT->defined()) dnc = f32c(*dnT);
  auto fo = q.options().dtype(at::kFloat);
  Tensor dq = at::empty_like(q), dk = at::empty_like(k), dv = at::empty_like(v);
  Tensor dc0 = at::empty({d.B, d.NH, d.DQ, d.DV}, fo), dn0 = at::empty({d.B, d.NH, d.DQ}, fo);
  Tensor qdq = at::empty({d.B, d.NH, d.T}, fo), kdk = at::empty({d.B, d.NH, d.T}, fo);
  sc_check(sc_mlstm_bwd(q.data_ptr(), k.data_ptr(), v.data_ptr(), dtype_code(q), ig.data_ptr<float>(),
                        fg.data_ptr<float>(), hc.data_ptr(), dh.data_ptr(),
                        (const float*)opt_ptr(dcc), (const float*)opt_ptr(dnc), cs.data_ptr(),
                        ns.data_ptr<float>(), ms.data_ptr<float>(), mrow.data_ptr<float>(),
                        den.data_ptr<float>(), (int)BH, (int)d.T, (int)d.DQ, (int)d.DV, (float)eps,
                        dc0.data_ptr<float>(), dn0.data_ptr<float>(), dq.data_ptr(), dk.data_ptr(),
                        dv.data_ptr(), qdq.data_ptr<float>(), kdk.data_ptr<float>(), nullptr,
                        stream_for(q)),
           "statecatcher::mlstm_bwd");
  return {dq, dk, dv, dc0, dn0, qdq, kdk};
}

std::tuple<Tensor, Tensor, Tensor, Tensor, Tensor, Tensor, Tensor> mlstm_bwd_meta(
    const Tensor& q, const Tensor& k, const Tensor& v, const Tensor& ig, const Tensor& fg,
    const Tensor& h, const Tensor& dh, const optional<Tensor>& dcT, const optional<Tensor>& dnT,
    const Tensor& cs, const Tensor& ns, const Tensor& ms, const Tensor& mrow, const Tensor& den,
    double eps) {
  const MlstmDims d = check_mlstm(q, k, v, ig, fg);
  auto fo = q.options().dtype(at::kFloat);
  return {at::empty(q.sizes(), q.options()), at::empty(k.sizes(), k.options()),
          at::empty(v.sizes(), v.options()), at::empty({d.B, d.NH, d.DQ, d.DV}, fo),
          at::empty({d.B, d.NH, d.DQ}, fo), at::empty({d.B, d.NH, d.T}, fo),
          at::empty({d.B, d.NH, d.T}, fo)};
}

// d fgate = sigmoid(-fgate) * (reverse cumulative sum of qdq - kdk) over the last dim [.., T]
Tensor mlstm_gate_bwd_hip(const Tensor& qdq_in, const Tensor& kdk_in, const Tensor& fg_in) {
  c10::DeviceGuard guard(qdq_in.device());
  TORCH_CHECK(qdq_in.sizes() == kdk_in.sizes() && kdk_in.sizes() == fg_in.sizes() &&
                  qdq_in.dim() >= 1 && qdq_in.size(-1) % 64 == 0,
              "statecatcher::mlstm_gate_bwd: qdq / kdk / fgate [.., T], T % 64 == 0");
  Tensor qdq = f32c(qdq_in), kdk = f32c(kdk_in), fg = f32c(fg_in);
  Tensor dfg = at::empty_like(qdq);
  const int64_t T = qdq.size(-1), BH = T ? qdq.numel() / T : 0;
  sc_check(sc_mlstm_gate_bwd(qdq.data_ptr<float>(), kdk.data_ptr<float>(), fg.data_ptr<float>(),
                             (int)BH, (int)T, dfg.data_ptr<float>(), nullptr, nullptr, 0, 0, 0, 0,
                             0.0f, stream_for(qdq)),
           "statecatcher::mlstm_gate_bwd");
  return dfg;
}

Tensor mlstm_gate_bwd_meta(const Tensor& qdq, const Tensor& kdk, const Tensor& fg) {
  TORCH_CHECK(qdq.sizes() == kdk.sizes() && kdk.sizes() == fg.sizes(),
              "statecatcher::mlstm_gate_bwd: shapes");
  return at::empty(qdq.sizes(), qdq.options().dtype(at::kFloat));
}

// ------------------------------------------------------------------- fused RNN-T joiner ------
// enc_p [B,T,J], pred_p [B,U+1,J] (the joiner's enc_proj / pred_proj outputs), W [V,J], bias
// [V]: RNNTPredictorJoiner's joint + log_softmax + warp_rnnt's gathered lattice
// (model.py:73-145) without the (B,T,U+1,V) logits.
void check_joint(const Tensor& enc, const Tensor& pred, const Tensor& W, const Tensor& bias,
                 const Tensor& labels) {
  TORCH_CHECK(enc.dim() == 3 && pred.dim() == 3 && pred.size(0) == enc.size(0) &&
                  pred.size(2) == enc.size(2) && W.dim() == 2 && W.size(1) == enc.size(2) &&
                  bias.dim() == 1 && bias.size(0) == W.size(0),
              "statecatcher::rnnt_joint: enc_p [B,T,J], pred_p [B,U+1,J], W [V,J], bias [V]");
  TORCH_CHECK(labels.dim() == 2 && labels.size(0) == enc.size(0) && labels.size(1) >= pred.size(1) - 1,
              "statecatcher::rnnt_joint: labels must be padded [B, >= U]");
}

std::tuple<Tensor, Tensor> rnnt_joint_fwd_hip(const Tensor& enc_in, const Tensor& pred_in,
                                              const Tensor& W_in, const Tensor& bias_in,
                                              const Tensor& labels_in, const Tensor& flen_in,
                                              const Tensor& llen_in, int64_t blank) {
  c10::DeviceGuard guard(enc_in.device());
  check_joint(enc_in, pred_in, W_in, bias_in, labels_in);
  Tensor enc = f32c(enc_in), pred = f32c(pred_in), bias = f32c(bias_in);
  Tensor W = W_in.to(at::kBFloat16).contiguous();
  const int64_t B = enc.size(0), T = enc.size(1), J = enc.size(2), U = pred.size(1) - 1, V = W.size(0);
  Tensor labels = labels_in.to(at::kLong).narrow(1, 0, U).contiguous();
  Tensor flen = flen_in.to(at::kLong).contiguous(), llen = llen_in.to(at::kLong).contiguous();
  const int64_t wsb = (int64_t)sc_rnnt_workspace_bytes((int)B, (int)std::max<int64_t>(T, 1), (int)U);
  Tensor ws = at::empty({wsb}, enc.options().dtype(at::kByte));
  Tensor nll = at::empty({B}, enc.options());
  if (T == 0 || B == 0) {
    nll.fill_(std::numeric_limits<double>::infinity());
    return {nll, ws};
  }
  sc_check(sc_rnnt_joint_fwd(enc.data_ptr<float>(), pred.data_ptr<float>(), W.data_ptr(),
                             bias.data_ptr<float>(), (int)B, (int)T, (int)U, (int)V, (int)J,
                             labels.data_ptr<int64_t>(), U ? labels.stride(0) : 0,
                             flen.data_ptr<int64_t>(), llen.data_ptr<int64_t>(), (int)blank,
                             nll.data_ptr<float>(), ws.data_ptr(), (size_t)wsb, stream_for(enc)),
           "statecatcher::rnnt_joint_fwd");
  return {nll, ws};
}

std::tuple<Tensor, Tensor> rnnt_joint_fwd_meta(const Tensor& enc, const Tensor& pred, const Tensor& W,
                                               const Tensor& bias, const Tensor& labels,
                                               const Tensor& flen, const Tensor& llen, int64_t blank) {
  check_joint(enc, pred, W, bias, labels);
  const int64_t wsb = (int64_t)sc_rnnt_workspace_bytes(
      (int)enc.size(0), (int)std::max<int64_t>(enc.size(1), 1), (int)(pred.size(1) - 1));
  return {at::empty({enc.size(0)}, enc.options().dtype(at::kFloat)),
          at::empty({wsb}, enc.options().dtype(at::kByte))};
}

Tensor colsum_rows(const Tensor& x2d) {   // fixed-order fp32 column sums (sc_colsum)
  const int64_t M = x2d.size(0), N = x2d.size(1);
  Tensor out = at::empty({N}, x2d.options().dtype(at::kFloat));
  const size_t wsb = sc_colsum_workspace_bytes((int)M, (int)N);
  Tensor ws = at::empty({(int64_t)wsb}, x2d.options().dtype(at::kByte));
  sc_check(sc_colsum(x2d.data_ptr(), dtype_code(x2d), (int)M, (int)N, x2d.stride(0), 1, 1,
                     out.data_ptr<float>(), ws.data_ptr(), wsb, stream_for(x2d)),
           "statecatcher::colsum");
  return out;
}

std::tuple<Tensor, Tensor, Tensor, Tensor> rnnt_joint_bwd_hip(
    const Tensor& enc_in, const Tensor& pred_in, const Tensor& W_in, const Tensor& bias_in,
    const Tensor& labels_in, const Tensor& flen_in, const Tensor& llen_in, const Tensor& ws,
    const Tensor& scale_in, int64_t blank) {
  c10::DeviceGuard guard(enc_in.device());
  check_joint(enc_in, pred_in, W_in, bias_in, labels_in);
  Tensor enc = f32c(enc_in), pred = f32c(pred_in), bias = f32c(bias_in);
  Tensor W = W_in.to(at::kBFloat16).contiguous();
  const int64_t B = enc.size(0), T = enc.size(1), J = enc.size(2), U = pred.size(1) - 1, V = W.size(0);
  Tensor labels = labels_in.to(at::kLong).narrow(1, 0, U).contiguous();
  Tensor flen = flen_in.to(at::kLong).contiguous(), llen = llen_in.to(at::kLong).contiguous();
  auto fo = enc.options();
  if (T == 0 || B == 0)
    return {at::zeros_like(enc), at::zeros_like(pred), at::zeros({V, J}, fo), at::zeros({V}, fo)};
  int ntb = 0, nus = 0, S = 0;
  sc_check(sc_rnnt_joint_geometry((int)B, (int)T, (int)U, (int)V, &ntb, &nus, &S),
           "statecatcher::rnnt_joint_geometry");
  Tensor d_enc = at::empty({nus, B, T, J}, fo), d_pred = at::zeros({B, ntb, U + 1, J}, fo);
  Tensor dW = at::empty({S, V, J}, fo), db = at::empty({S, V}, fo);
  Tensor scale = f32c(scale_in.expand({B}));
  sc_check(sc_rnnt_joint_bwd(enc.data_ptr<float>(), pred.data_ptr<float>(), W.data_ptr(),
                             bias.data_ptr<float>(), (int)B, (int)T, (int)U, (int)V, (int)J,
                             labels.data_ptr<int64_t>(), U ? labels.stride(0) : 0,
                             flen.data_ptr<int64_t>(), llen.data_ptr<int64_t>(), (int)blank,
                             scale.data_ptr<float>(), d_enc.data_ptr<float>(), d_pred.data_ptr<float>(),
                             dW.data_ptr<float>(), db.data_ptr<float>(), ws.data_ptr(),
                             (size_t)ws.numel(), stream_for(enc)),
           "statecatcher::rnnt_joint_bwd");
  return {d_enc.sum(0), d_pred.sum(1), colsum_rows(dW.view({S, V * J})).view({V, J}), colsum_rows(db)};
}

std::tuple<Tensor, Tensor, Tensor, Tensor> rnnt_joint_bwd_meta(
    const Tensor& enc, const Tensor& pred, const Tensor& W, const Tensor& bias, const Tensor& labels,
    const Tensor& flen, const Tensor& llen, const Tensor& ws, const Tensor& scale, int64_t blank) {
  check_joint(enc, pred, W, bias, labels);
  auto fo = enc.options().dtype(at::kFloat);
  return {at::empty(enc.sizes(), fo), at::empty(pred.sizes(), fo), at::empty(W.sizes(), fo),
          at::empty(bias.sizes(), fo)};
}

// ------------------------------------------------------------------- projection GEMMs ------
// C [M,N] bf16 = a [M,K] b [N,K]^T on the persistent MFMA kernel (sc_gemm_tn_bf16)
Tensor gemm_tn_hip(const Tensor& a_in, const Tensor& b_in, int64_t tile_m) {
  c10::DeviceGuard guard(a_in.device());
  TORCH_CHECK(a_in.dim() == 2 && b_in.dim() == 2 && a_in.size(1) == b_in.size(1) &&
                  a_in.scalar_type() == at::kBFloat16 && b_in.scalar_type() == at::kBFloat16,
              "statecatcher::gemm_tn: a [M,K], b [N,K] bfloat16");
  Tensor a = a_in.contiguous(), b = b_in.contiguous();
  const int64_t M = a.size(0), N = b.size(0), K = a.size(1);
  Tensor c = at::empty({M, N}, a.options());
  if (M == 0 || N == 0) return c;
  sc_check(sc_gemm_tn_bf16(a.data_ptr(), K, b.data_ptr(), K, c.data_ptr(), N, (int)M, (int)N,
                           (int)K, (int)tile_m, stream_for(a)),
           "statecatcher::gemm_tn");
  return c;
}

Tensor gemm_tn_meta(const Tensor& a, const Tensor& b, int64_t tile_m) {
  TORCH_CHECK(a.dim() == 2 && b.dim() == 2 && a.size(1) == b.size(1), "statecatcher::gemm_tn: shapes");
  return at::empty({a.size(0), b.size(0)}, a.options());
}

// dW [N,K] fp32 = dy [M,N]^T x [M,K] (bf16 operands): the split-L MFMA kernel
// (sc_gemm_wgrad_bf16) and the fixed-order slab sum (sc_colsum); block_d = D > 0: dy's columns
// are in step-blocked gate order and dW comes back in the reference's row order
Tensor gemm_wgrad_hip(const Tensor& dy_in, const Tensor& x_in, int64_t block_d) {
  c10::DeviceGuard guard(dy_in.device());
  TORCH_CHECK(dy_in.dim() == 2 && x_in.dim() == 2 && dy_in.size(0) == x_in.size(0) &&
                  dy_in.scalar_type() == at::kBFloat16 && x_in.scalar_type() == at::kBFloat16,
              "statecatcher::gemm_wgrad: dy [M,N], x [M,K] bfloat16");
  Tensor dy = dy_in.contiguous(), x = x_in.contiguous();
  const int64_t M = dy.size(0), N = dy.size(1), K = x.size(1);
  TORCH_CHECK(block_d == 0 || (N == 7 * block_d && block_d % 64 == 0),
              "statecatcher::gemm_wgrad: block_d must be 0 or N / 7 (a multiple of 64)");
  const int S = sc_gemm_wgrad_splits((int)M, (int)N, (int)K);
  TORCH_CHECK(S > 0, "statecatcher::gemm_wgrad: shape [", M, ",", N, "] x [", M, ",", K,
              "] outside the MFMA kernel's tiling (sc_gemm_wgrad_splits == 0)");
  Tensor part = at::empty({S, N, K}, dy.options().dtype(at::kFloat));
  void* st = stream_for(dy);
  sc_check(sc_gemm_wgrad_bf16(dy.data_ptr(), N, x.data_ptr(), K, part.data_ptr<float>(), (int)M,
                              (int)N, (int)K, S, st),
           "statecatcher::gemm_wgrad");
  Tensor dw = at::empty({N, K}, part.options());
  const size_t wsb = sc_colsum_workspace_bytes(S, N * K);
  Tensor ws = at::empty({(int64_t)wsb}, dy.options().dtype(at::kByte));
  sc_check(sc_colsum(part.data_ptr(), SC_F32, S, N * K, N * K, block_d ? block_d / 64 : 1,
                     block_d ? 7 : 1, dw.data_ptr<float>(), ws.data_ptr(), wsb, st),
           "statecatcher::gemm_wgrad (slab sum)");
  return dw;
}

Tensor gemm_wgrad_meta(const Tensor& dy, const Tensor& x, int64_t block_d) {
  TORCH_CHECK(dy.dim() == 2 && x.dim() == 2 && dy.size(0) == x.size(0), "statecatcher::gemm_wgrad: shapes");
  return at::empty({dy.size(1), x.size(1)}, dy.options().dtype(at::kFloat));
}

// --------------------------------------------------------------------- optimizer step ------
// clip_grad_norm_(clipped tensors, max_norm) then Adam / AdamW on every tensor, in place on
// params / exp_avgs / exp_avg_sqs (torch's own optimizer state); grads are read only.  The first
// n_clip tensors form the clip set (the reference clips model.parameters() only).  Returns the
// total norm clip_grad_norm_ reports (0-dim fp32; 0 when max_norm <= 0: no clipping).
Tensor clip_adam_hip(at::TensorList params, at::TensorList grads, at::TensorList exp_avgs,
                     at::TensorList exp_avg_sqs, int64_t n_clip, double max_norm, double lr,
                     double beta1, double beta2, double eps, double weight_decay, bool decoupled,
                     double step_size, double bc2_sqrt) {
  const size_t nt = params.size();
  TORCH_CHECK(nt > 0 && grads.size() == nt && exp_avgs.size() == nt && exp_avg_sqs.size() == nt,
              "statecatcher::clip_adam_: equal-length tensor lists");
  TORCH_CHECK(n_clip >= 0 && n_clip <= (int64_t)nt, "statecatcher::clip_adam_: n_clip");
  c10::DeviceGuard guard(params[0].device());
  std::vector<sc_adam_tensor> t(nt);
  for (size_t i = 0; i < nt; ++i) {
    for (const Tensor* x : {&params[i], &grads[i], &exp_avgs[i], &exp_avg_sqs[i]})
      TORCH_CHECK(x->is_cuda() && x->scalar_type() == at::kFloat && x->is_contiguous() &&
                      x->numel() == params[i].numel() && x->device() == params[0].device(),
                  "statecatcher::clip_adam_: fp32 contiguous tensors of equal size, all on the "
                  "device of params[0]");
    t[i] = sc_adam_tensor{params[i].data_ptr<float>(), grads[i].data_ptr<float>(),
                          exp_avgs[i].data_ptr<float>(), exp_avg_sqs[i].data_ptr<float>(),
                          params[i].numel()};
  }
  void* st = stream_for(params[0]);
  Tensor norm = at::zeros({}, params[0].options());
  Tensor part;
  int64_t np = 0;
  if (max_norm > 0.0 && n_clip > 0) {
    np = sc_adam_parts(t.data(), (int)n_clip);
    part = at::empty({np}, params[0].options());
    sc_check(sc_adam_sumsq(t.data(), (int)n_clip, part.data_ptr<float>(), st),
             "statecatcher::clip_adam_ (sum of squares)");
  }
  // the clipped tensors with the clip coefficient, then the rest unclipped
  sc_check(sc_adam_step(t.data(), (int)n_clip, np ? part.data_ptr<float>() : nullptr, np,
                        max_norm, lr, beta1, beta2, eps, weight_decay, decoupled ? 1 : 0,
                        step_size, bc2_sqrt, np ? norm.data_ptr<float>() : nullptr, st),
           "statecatcher::clip_adam_");
  if ((int64_t)nt > n_clip)
    sc_check(sc_adam_step(t.data() + n_clip, (int)(nt - n_clip), nullptr, 0, max_norm, lr, beta1,
                          beta2, eps, weight_decay, decoupled ? 1 : 0, step_size, bc2_sqrt,
                          nullptr, st),
             "statecatcher::clip_adam_ (unclipped)");
  return norm;
}

Tensor clip_adam_meta(at::TensorList params, at::TensorList grads, at::TensorList exp_avgs,
                      at::TensorList exp_avg_sqs, int64_t n_clip, double max_norm, double lr,
                      double beta1, double beta2, double eps, double weight_decay, bool decoupled,
                      double step_size, double bc2_sqrt) {
  TORCH_CHECK(!params.empty(), "statecatcher::clip_adam_: empty parameter list");
  return at::empty({}, params[0].options());
}

}  // namespace


TORCH_LIBRARY(statecatcher, m) {
  m.def("abi_version() -> int", []() -> int64_t { return sc_abi_version(); });
  m.def("lucy_scan_fwd(Tensor gates, Tensor h0, Tensor s0, Tensor? gate_bias=None, bool need_ckpt=True)"
        " -> (Tensor out, Tensor s_last, Tensor h_last, Tensor ckpt)");
  m.def("lucy_scan_bwd(Tensor gates, Tensor ckpt, Tensor dout, Tensor? ds_last=None, "
        "Tensor? gate_bias=None, bool want_dbias=False) -> (Tensor dgates, Tensor dh0, Tensor ds0, "
        "Tensor dbias)");
  m.def("decay_scan_fwd(Tensor kv, Tensor decay, Tensor? init=None) -> Tensor");
  m.def("decay_scan_bwd(Tensor decay, Tensor s_all, Tensor dout, Tensor? init=None)"
        " -> (Tensor dkv, Tensor ddecay, Tensor dinit)");
  m.def("layer_norm_fwd(Tensor x, Tensor gamma, Tensor beta, float eps=1e-5)"
        " -> (Tensor y, Tensor mean, Tensor rstd)");
  m.def("layer_norm_bwd(Tensor x, Tensor dy, Tensor gamma, Tensor mean, Tensor rstd)"
        " -> (Tensor dx, Tensor dgamma, Tensor dbeta)");
  m.def("ctc_fwd(Tensor x, Tensor targets, Tensor in_lens, Tensor tgt_lens, int blank=0, "
        "bool is_logits=True) -> (Tensor nll, Tensor workspace)");
  m.def("ctc_bwd(Tensor x, Tensor targets, Tensor in_lens, Tensor tgt_lens, Tensor nll, "
        "Tensor workspace, Tensor scale, int blank=0, bool is_logits=True) -> Tensor");
  m.def("ctc_mean(Tensor nll, Tensor tgt_lens) -> (Tensor loss, Tensor factor)");
  m.def("ctc_greedy_decode(Tensor log_probs, Tensor lengths, int blank=0)"
        " -> (Tensor tokens, Tensor counts)");
  m.def("mlstm_fwd(Tensor q, Tensor k, Tensor v, Tensor igate, Tensor fgate, Tensor? c0=None, "
        "Tensor? n0=None, Tensor? m0=None, float eps=1e-6) -> (Tensor h, Tensor c_last, "
        "Tensor n_states, Tensor m_states, Tensor c_states, Tensor m_rows, Tensor den_rows)");
  m.def("mlstm_bwd(Tensor q, Tensor k, Tensor v, Tensor igate, Tensor fgate, Tensor h, Tensor dh, "
        "Tensor? dc_last, Tensor? dn_last, Tensor c_states, Tensor n_states, Tensor m_states, "
        "Tensor m_rows, Tensor den_rows, float eps=1e-6) -> (Tensor dq, Tensor dk, Tensor dv, "
        "Tensor dc0, Tensor dn0, Tensor qdq, Tensor kdk)");
  m.def("mlstm_gate_bwd(Tensor qdq, Tensor kdk, Tensor fgate) -> Tensor");
  m.def("rnnt_joint_fwd(Tensor enc_p, Tensor pred_p, Tensor W, Tensor bias, Tensor labels, "
        "Tensor frames_lengths, Tensor labels_lengths, int blank=0) -> (Tensor nll, Tensor workspace)");
  m.def("gemm_tn(Tensor a, Tensor b, int tile_m=0) -> Tensor");
  m.def("gemm_wgrad(Tensor dy, Tensor x, int block_d=0) -> Tensor");
  m.def("clip_adam_(Tensor(a!)[] params, Tensor[] grads, Tensor(b!)[] exp_avgs, "
        "Tensor(c!)[] exp_avg_sqs, int n_clip, float max_norm, float lr, float beta1, float beta2, "
        "float eps, float weight_decay, bool decoupled, float step_size, float bc2_sqrt) -> Tensor");
  m.def("rnnt_joint_bwd(Tensor enc_p, Tensor pred_p, Tensor W, Tensor bias, Tensor labels, "
        "Tensor frames_lengths, Tensor labels_lengths, Tensor workspace, Tensor scale, int blank=0)"
        " -> (Tensor d_enc, Tensor d_pred, Tensor dW, Tensor dbias)");
}

TORCH_LIBRARY_IMPL(statecatcher, CUDA, m) {
  m.impl("lucy_scan_fwd", &lucy_scan_fwd_hip);
  m.impl("lucy_scan_bwd", &lucy_scan_bwd_hip);
  m.impl("decay_scan_fwd", &decay_scan_fwd_hip);
  m.impl("decay_scan_bwd", &decay_scan_bwd_hip);
  m.impl("layer_norm_fwd", &layer_norm_fwd_hip);
  m.impl("layer_norm_bwd", &layer_norm_bwd_hip);
  m.impl("ctc_fwd", &ctc_fwd_hip);
  m.impl("ctc_bwd", &ctc_bwd_hip);
  m.impl("ctc_mean", &ctc_mean_hip);
  m.impl("ctc_greedy_decode", &ctc_greedy_decode_hip);
  m.impl("mlstm_fwd", &mlstm_fwd_hip);
  m.impl("mlstm_bwd", &mlstm_bwd_hip);
  m.impl("mlstm_gate_bwd", &mlstm_gate_bwd_hip);
  m.impl("rnnt_joint_fwd", &rnnt_joint_fwd_hip);
  m.impl("rnnt_joint_bwd", &rnnt_joint_bwd_hip);
  m.impl("gemm_tn", &gemm_tn_hip);
  m.impl("gemm_wgrad", &gemm_wgrad_hip);
  m.impl("clip_adam_", &clip_adam_hip);
}

TORCH_LIBRARY_IMPL(statecatcher, Meta, m) {
  m.impl("lucy_scan_fwd", &lucy_scan_fwd_meta);
  m.impl("lucy_scan_bwd", &lucy_scan_bwd_meta);
  m.impl("decay_scan_fwd", &decay_scan_fwd_meta);
  m.impl("decay_scan_bwd", &decay_scan_bwd_meta);
  m.impl("layer_norm_fwd", &layer_norm_fwd_meta);
  m.impl("layer_norm_bwd", &layer_norm_bwd_meta);
  m.impl("ctc_fwd", &ctc_fwd_meta);
  m.impl("ctc_bwd", &ctc_bwd_meta);
  m.impl("ctc_mean", &ctc_mean_meta);
  m.impl("ctc_greedy_decode", &ctc_greedy_decode_meta);
  m.impl("mlstm_fwd", &mlstm_fwd_meta);
  m.impl("mlstm_bwd", &mlstm_bwd_meta);
  m.impl("mlstm_gate_bwd", &mlstm_gate_bwd_meta);
  m.impl("rnnt_joint_fwd", &rnnt_joint_fwd_meta);
  m.impl("rnnt_joint_bwd", &rnnt_joint_bwd_meta);
  m.impl("gemm_tn", &gemm_tn_meta);
  m.impl("gemm_wgrad", &gemm_wgrad_meta);
  m.impl("clip_adam_", &clip_adam_meta);
}
