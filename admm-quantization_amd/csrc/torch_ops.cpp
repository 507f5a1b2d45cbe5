// PyTorch custom operators (torch.ops.admmq.*) over the C-ABI of libadmmq.so.
//
// The Python drop-ins (admmq.admm / .quantization / .als) call these ops; each op
// validates its tensors, allocates the caller-owned workspace through PyTorch's
// caching allocator, and calls the same stream-ordered entry points of
// include/admmq.h on the current HIP stream. Reference interfaces mirrored:
//   admmq::admm_iteration_batched  <- source/admm.py:51-67 admm_iteration (batched over problems)
//   admmq::quantize_batched        <- source/quantization.py:69-144 quantize_tensor
//   admmq::quantize_channel        <- source/quantization.py:29-33, 91-106 (channel_* schemes with a dim)
//   admmq::cp_gram_mttkrp          <- scripts/factorize.py:215-237 / :276-287 (G, F of one mode)
//   admmq::cp_rel_error            <- scripts/factorize.py:246-253 + source/admm.py:14-15
// Registered for the CUDA dispatch key (HIP tensors on ROCm builds of PyTorch), with
// Meta kernels for shape propagation (fake tensors / torch.compile tracing). There is
// no CPU kernel: CPU tensors fail in the dispatcher.
#include <torch/library.h>
#include <ATen/ATen.h>
#include <c10/hip/HIPStream.h>
#include <c10/core/DeviceGuard.h>
#include <c10/util/Exception.h>

#include <atomic>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/admmq.h"

namespace {

void check_rc(int32_t rc, const char* what) {
  TORCH_CHECK(rc == ADMMQ_OK, "admmq: ", what, " failed (status ", rc, "): ", admmq_last_error());
}

void check_f32_device(const at::Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda(), "admmq: ", name, " must live on a ROCm GPU (the MI355X path has no CPU implementation)");
  TORCH_CHECK(t.scalar_type() == at::kFloat, "admmq: ", name, " must be float32, got ", t.scalar_type());
}

// every tensor of a call on one device: the workspace, the stream and the launches use it
void check_same_device(const at::Tensor& t, const at::Tensor& ref, const char* name) {
  TORCH_CHECK(t.device() == ref.device(), "admmq: ", name, " is on ", t.device(), " but the call's first tensor is on ",
              ref.device());
}

void* stream_of(const at::Tensor& t) {
  return static_cast<void*>(c10::hip::getCurrentHIPStream(t.device().index()).stream());
}

at::Tensor workspace(size_t nbytes, const at::Tensor& like) {
  return at::empty({static_cast<int64_t>(std::max<size_t>(nbytes, 256))}, like.options().dtype(at::kByte));
}

// Calls whose internal fault was repaired by a re-run (check_fault), process-wide:
// admmq::fault_repairs (expected 0 on an undisturbed device)
std::atomic<int64_t> g_fault_repairs{0};
int64_t fault_repairs(bool reset) { return reset ? g_fault_repairs.exchange(0) : g_fault_repairs.load(); }

// --- admm_iteration_batched -------------------------------------------------------
// solve: -1 = the process default (admmq_set_solve_mode; fp32 unless changed), else
// ADMMQ_SOLVE_FP32 / ADMMQ_SOLVE_SPLIT for this call.
// check_fault (default): the call syncs once at its end to read the internal-fault column
// of `info`: when the fused finalize's bounded wait timed out somewhere (its launch's
// blocks were not all resident), the call restores U and re-runs with the separate
// finalize launch, so it never returns unfinalized factors (same results as an
// undisturbed run). check_fault = false: no sync; the caller must check info[:, 3]
// itself and repeat the call (with U restored) where it is nonzero. The returned info is
// [n, 5]: the C-ABI's {iterations run, converged, spd_error, internal fault} plus the
// re-runs this call made (0, or 1 after a repaired fault; also counted in fault_repairs).
std::tuple<std::vector<at::Tensor>, at::Tensor, std::vector<at::Tensor>, std::vector<at::Tensor>> admm_batched_cuda(
    at::TensorList H, at::TensorList U, at::TensorList F, at::TensorList G, int64_t max_iter, double eps,
    int64_t bits, int64_t qscheme, int64_t num_attempts, bool check_spd, bool debug, int64_t solve,
    bool check_fault) {
  const size_t n = H.size();
  TORCH_CHECK(n > 0, "admmq: admm_iteration_batched needs at least one problem");
  TORCH_CHECK(U.size() == n && F.size() == n && G.size() == n, "admmq: H, U, F, G lists differ in length");
  check_f32_device(H[0], "H");
  const c10::DeviceGuard guard(H[0].device());
  std::vector<at::Tensor> Hc, Uc, Fc, Gc, outs, hts, xs;
  std::vector<admmq_problem> probs(n);
  for (size_t i = 0; i < n; ++i) {
    check_f32_device(H[i], "H"); check_f32_device(U[i], "U"); check_f32_device(F[i], "F"); check_f32_device(G[i], "G");
    check_same_device(H[i], H[0], "H"); check_same_device(U[i], H[0], "U");
    check_same_device(F[i], H[0], "F"); check_same_device(G[i], H[0], "G");
    TORCH_CHECK(H[i].dim() == 2, "admm_iteration expects 2-D factors (I, R)");
    const int64_t I = H[i].size(0), R = H[i].size(1);
    TORCH_CHECK(F[i].sizes() == H[i].sizes() && U[i].sizes() == H[i].sizes() && G[i].dim() == 2 &&
                    G[i].size(0) == R && G[i].size(1) == R,
                "admm_iteration: shape mismatch H", H[i].sizes(), " U", U[i].sizes(), " F", F[i].sizes(), " G",
                G[i].sizes());
    Hc.push_back(H[i].contiguous()); Uc.push_back(U[i].contiguous());
    Fc.push_back(F[i].contiguous()); Gc.push_back(G[i].contiguous());
    outs.push_back(at::empty_like(Hc.back()));
    if (debug) { hts.push_back(at::empty_like(Hc.back())); xs.push_back(at::empty_like(Hc.back())); }
    admmq_problem& p = probs[i];
    p.F = Fc.back().data_ptr<float>(); p.G = Gc.back().data_ptr<float>(); p.H0 = Hc.back().data_ptr<float>();
    p.H_out = outs.back().data_ptr<float>(); p.U = Uc.back().data_ptr<float>();
    p.HT_out = debug ? hts.back().data_ptr<float>() : nullptr;
    p.X_out = debug ? xs.back().data_ptr<float>() : nullptr;
    p.I = static_cast<int32_t>(I); p.R = static_cast<int32_t>(R);
  }
  admmq_admm_options opt;
  check_rc(admmq_admm_default_options(&opt), "default_options");
  if (solve >= 0) opt.solve_mode = static_cast<int32_t>(solve);
  const at::Tensor& ref = Hc[0];
  void* stream = stream_of(ref);
  const int32_t nn = static_cast<int32_t>(n);
  const int32_t na = static_cast<int32_t>(num_attempts);
  const size_t nb = admmq_admm_workspace_size_ex(probs.data(), nn, na, &opt);
  TORCH_CHECK(nb != 0, "admmq: admm workspace planning failed: ", admmq_last_error());
  at::Tensor ws = workspace(nb, ref);
  at::Tensor info5 = at::zeros({nn, 5}, ref.options().dtype(at::kInt));
  at::Tensor info = at::zeros({nn, 4}, ref.options().dtype(at::kInt));   // the C-ABI's int32[nprob * 4]
  check_rc(admmq_admm_prepare_ex(probs.data(), nn, na, &opt, ws.data_ptr(), ws.numel(), stream), "admm_prepare");
  if (check_spd || max_iter <= 1) {
    // source/admm.py:54 raises before anything is modified: one sync per call
    check_rc(admmq_admm_run_ex(probs.data(), nn, 1, 0.f, 4, 0, na, &opt, ws.data_ptr(), ws.numel(),
                               info.data_ptr<int32_t>(), stream),
             "admm_info");
    TORCH_CHECK_LINALG(info.select(1, 2).max().item<int32_t>() == 0,
                       "linalg.cholesky: The factorization could not be completed because the input is not "
                       "positive-definite.");
  }
  auto info_out = [&](int64_t reruns) {
    info5.narrow(1, 0, 4).copy_(info);
    if (reruns) info5.select(1, 4).fill_(reruns);
    return info5;
  };
  if (max_iter <= 1) {   // the reference returns H unchanged (the Python drop-in returns the caller's object)
    std::vector<at::Tensor> same;
    for (const at::Tensor& h : H) same.push_back(h.clone());
    return {same, info_out(0), hts, xs};
  }
  std::vector<at::Tensor> ubak;   // U before the run: restored if the run must be repeated
  if (check_fault)
    for (const at::Tensor& u : Uc) ubak.push_back(u.clone());
  auto run = [&]() {
    check_rc(admmq_admm_run_ex(probs.data(), nn, static_cast<int32_t>(max_iter), static_cast<float>(eps),
                               static_cast<int32_t>(bits), static_cast<int32_t>(qscheme), na, &opt, ws.data_ptr(),
                               ws.numel(), info.data_ptr<int32_t>(), stream),
             "admm_run");
  };
  run();
  int64_t reruns = 0;
  if (check_fault && info.select(1, 3).max().item<int32_t>() != 0) {   // internal fault: repeat without the fused finalize
    for (size_t i = 0; i < n; ++i) Uc[i].copy_(ubak[i]);
    opt.fused_finalize = 0;
    check_rc(admmq_admm_prepare_ex(probs.data(), nn, na, &opt, ws.data_ptr(), ws.numel(), stream), "admm_prepare");
    run();
    TORCH_CHECK(info.select(1, 3).max().item<int32_t>() == 0, "admmq: internal fault in the separate-finalize re-run");
    reruns = 1;
    g_fault_repairs.fetch_add(1);
  }
  for (size_t i = 0; i < n; ++i)   // U is updated in place (source/admm.py:60)
    if (!U[i].is_same(Uc[i])) const_cast<at::Tensor&>(U[i]).copy_(Uc[i]);
  return {outs, info_out(reruns), hts, xs};
}

std::tuple<std::vector<at::Tensor>, at::Tensor, std::vector<at::Tensor>, std::vector<at::Tensor>> admm_batched_meta(
    at::TensorList H, at::TensorList U, at::TensorList F, at::TensorList G, int64_t max_iter, double eps,
    int64_t bits, int64_t qscheme, int64_t num_attempts, bool check_spd, bool debug, int64_t solve,
    bool check_fault) {
  std::vector<at::Tensor> outs, hts, xs;
  for (const at::Tensor& h : H) {
    outs.push_back(at::empty_like(h));
    if (debug) { hts.push_back(at::empty_like(h)); xs.push_back(at::empty_like(h)); }
  }
  const int64_t n = static_cast<int64_t>(H.size());
  return {outs, at::empty({n, 5}, H[0].options().dtype(at::kInt)), hts, xs};
}

// --- quantize_batched ----------------------------------------------------------------
std::vector<at::Tensor> quantize_batched_cuda(at::TensorList x, int64_t bits, int64_t qscheme, int64_t num_attempts,
                                              std::optional<double> tmin, std::optional<double> tmax) {
  TORCH_CHECK(!x.empty(), "admmq: quantize_batched needs at least one tensor");
  TORCH_CHECK(bits >= 1, "admmq: bits must be >= 1");
  check_f32_device(x[0], "tensor");
  const c10::DeviceGuard guard(x[0].device());
  const bool has_kw = qscheme == ADMMQ_TENSOR_AFFINE && tmin.has_value() && tmax.has_value();
  std::vector<at::Tensor> xs, ys;
  std::vector<admmq_qtensor> items(x.size());
  for (size_t i = 0; i < x.size(); ++i) {
    check_f32_device(x[i], "tensor");
    check_same_device(x[i], x[0], "tensor");
    TORCH_CHECK(x[i].numel() > 0, "min(): Expected reduction dim to be specified for input.numel() == 0.");
    xs.push_back(x[i].contiguous());
    ys.push_back(at::empty_like(xs.back()));
    const int64_t cols = xs.back().dim() == 0 ? 1 : xs.back().size(-1);
    admmq_qtensor& t = items[i];
    t.x = xs.back().data_ptr<float>(); t.y = ys.back().data_ptr<float>();
    t.rows = xs.back().numel() / cols; t.cols = cols;
    t.tmin = has_kw ? static_cast<float>(*tmin) : 0.f; t.tmax = has_kw ? static_cast<float>(*tmax) : 0.f;
    t.has_minmax = has_kw ? 1 : 0; t.reserved = 0;
  }
  const int32_t n = static_cast<int32_t>(items.size());
  const size_t nb = admmq_quantize_workspace_size(items.data(), n, static_cast<int32_t>(num_attempts));
  TORCH_CHECK(nb != 0, "admmq: quantize workspace planning failed: ", admmq_last_error());
  at::Tensor ws = workspace(nb, xs[0]);
  check_rc(admmq_quantize_batched(items.data(), n, static_cast<int32_t>(bits), static_cast<int32_t>(qscheme),
                                  static_cast<int32_t>(num_attempts), ws.data_ptr(), ws.numel(), stream_of(xs[0])),
           "quantize_batched");
  return ys;
}

std::vector<at::Tensor> quantize_batched_meta(at::TensorList x, int64_t bits, int64_t qscheme, int64_t num_attempts,
                                              std::optional<double> tmin, std::optional<double> tmax) {
  std::vector<at::Tensor> ys;
  for (const at::Tensor& t : x) ys.push_back(at::empty_like(t, t.options().memory_format(at::MemoryFormat::Contiguous)));
  return ys;
}

// --- quantize_channel (channel_symmetric / channel_affine with an explicit dim) ----------------
at::Tensor quantize_channel_cuda(const at::Tensor& x, int64_t bits, int64_t qscheme, int64_t dim) {
  check_f32_device(x, "tensor");
  const c10::DeviceGuard guard(x.device());
  TORCH_CHECK(x.dim() >= 1, "admmq: quantize_channel needs a tensor with at least one dimension");
  TORCH_CHECK(x.numel() > 0, "min(): Expected reduction dim to be specified for input.numel() == 0.");
  const at::Tensor xc = x.contiguous();
  const int64_t nd = xc.dim();
  const int64_t d = dim < 0 ? dim + nd : dim;
  TORCH_CHECK_INDEX(d >= 0 && d < nd, "Dimension out of range (expected to be in range of [", -nd, ", ", nd - 1,
                    "], but got ", dim, ")");
  const int64_t C = xc.size(d), L = xc.size(nd - 1);
  TORCH_CHECK(L == C || L == 1 || C == 1, "The size of tensor a (", L, ") must match the size of tensor b (", C,
              ") at non-singleton dimension ", nd - 1);
  std::vector<int64_t> shape(xc.sizes().begin(), xc.sizes().end());
  std::vector<int64_t> oshape = shape;
  oshape[nd - 1] = std::max(L, C);
  at::Tensor y = at::empty(oshape, xc.options());
  const size_t nb = admmq_quantize_channel_workspace_size(shape.data(), static_cast<int32_t>(nd), static_cast<int32_t>(d));
  TORCH_CHECK(nb != 0, "admmq: quantize_channel planning failed: ", admmq_last_error());
  at::Tensor ws = workspace(nb, xc);
  check_rc(admmq_quantize_channel(xc.data_ptr<float>(), y.data_ptr<float>(), shape.data(), static_cast<int32_t>(nd),
                                  static_cast<int32_t>(d), static_cast<int32_t>(bits), static_cast<int32_t>(qscheme),
                                  ws.data_ptr(), ws.numel(), stream_of(xc)),
           "quantize_channel");
  return y;
}

at::Tensor quantize_channel_meta(const at::Tensor& x, int64_t bits, int64_t qscheme, int64_t dim) {
  const int64_t nd = x.dim();
  const int64_t d = dim < 0 ? dim + nd : dim;
  std::vector<int64_t> oshape(x.sizes().begin(), x.sizes().end());
  oshape[nd - 1] = std::max(x.size(nd - 1), x.size(d));
  return at::empty(oshape, x.options());
}

// --- ALS sweep contractions ---------------------------------------------------------------
// Layer l has tensor W[l] (2-D or 3-D) and factors[off_l .. off_l + W[l].dim()), off_l the
// running sum of the layers' dims.
std::vector<admmq_cp_layer> cp_layers(at::TensorList W, at::TensorList factors, std::vector<at::Tensor>& keep,
                                      std::vector<at::Tensor>* G, std::vector<at::Tensor>* F, int64_t mode) {
  std::vector<admmq_cp_layer> L(W.size());
  size_t off = 0;
  for (size_t l = 0; l < W.size(); ++l) {
    check_f32_device(W[l], "W");
    check_same_device(W[l], W[0], "W");
    const int64_t nd = W[l].dim();
    TORCH_CHECK(nd == 2 || nd == 3, "admmq: CP layer tensor must be 2-D or 3-D, got ", nd, "-D");
    TORCH_CHECK(off + nd <= factors.size(), "admmq: too few factors for the layers");
    keep.push_back(W[l].contiguous());
    admmq_cp_layer& c = L[l];
    c.W = keep.back().data_ptr<float>();
    const int64_t R = factors[off].size(1);
    for (int64_t d = 0; d < 3; ++d) {
      c.factors[d] = nullptr;
      c.dims[d] = d < nd ? static_cast<int32_t>(W[l].size(d)) : 0;
      if (d < nd) {
        const at::Tensor& f = factors[off + d];
        check_f32_device(f, "factor");
        check_same_device(f, W[0], "factor");
        TORCH_CHECK(f.dim() == 2 && f.size(0) == W[l].size(d) && f.size(1) == R, "admmq: factor ", d, " has shape ",
                    f.sizes(), ", expected (", W[l].size(d), ", ", R, ")");
        keep.push_back(f.contiguous());
        c.factors[d] = keep.back().data_ptr<float>();
      }
    }
    c.ndim = static_cast<int32_t>(nd);
    c.R = static_cast<int32_t>(R);
    c.G = nullptr; c.F = nullptr;
    if (G) {
      TORCH_CHECK(mode >= 0 && mode < nd, "admmq: mode ", mode, " out of range for a ", nd, "-way tensor");
      G->push_back(at::empty({R, R}, W[l].options()));
      F->push_back(at::empty({W[l].size(mode), R}, W[l].options()));
      c.G = G->back().data_ptr<float>();
      c.F = F->back().data_ptr<float>();
    }
    off += nd;
  }
  return L;
}

std::tuple<std::vector<at::Tensor>, std::vector<at::Tensor>> cp_gram_mttkrp_cuda(at::TensorList W,
                                                                                 at::TensorList factors, int64_t mode) {
  TORCH_CHECK(!W.empty(), "admmq: cp_gram_mttkrp needs at least one layer");
  check_f32_device(W[0], "W");
  const c10::DeviceGuard guard(W[0].device());
  std::vector<at::Tensor> keep, G, F;
  std::vector<admmq_cp_layer> L = cp_layers(W, factors, keep, &G, &F, mode);
  const int32_t n = static_cast<int32_t>(L.size());
  const size_t nb = admmq_cp_workspace_size(L.data(), n, static_cast<int32_t>(mode));
  TORCH_CHECK(nb != 0, "admmq: cp workspace planning failed: ", admmq_last_error());
  at::Tensor ws = workspace(nb, keep[0]);
  check_rc(admmq_cp_gram_mttkrp(L.data(), n, static_cast<int32_t>(mode), ws.data_ptr(), ws.numel(), stream_of(keep[0])),
           "cp_gram_mttkrp");
  return {G, F};
}

std::tuple<std::vector<at::Tensor>, std::vector<at::Tensor>> cp_gram_mttkrp_meta(at::TensorList W,
                                                                                 at::TensorList factors, int64_t mode) {
  std::vector<at::Tensor> G, F;
  size_t off = 0;
  for (const at::Tensor& w : W) {
    const int64_t R = factors[off].size(1);
    G.push_back(at::empty({R, R}, w.options()));
    F.push_back(at::empty({w.size(mode), R}, w.options()));
    off += w.dim();
  }
  return {G, F};
}

at::Tensor cp_rel_error_cuda(at::TensorList W, at::TensorList factors) {
  TORCH_CHECK(!W.empty(), "admmq: cp_rel_error needs at least one layer");
  check_f32_device(W[0], "W");
  const c10::DeviceGuard guard(W[0].device());
  std::vector<at::Tensor> keep;
  std::vector<admmq_cp_layer> L = cp_layers(W, factors, keep, nullptr, nullptr, 0);
  const int32_t n = static_cast<int32_t>(L.size());
  at::Tensor out = at::empty({n}, keep[0].options().dtype(at::kDouble));
  const size_t nb = admmq_cp_workspace_size(L.data(), n, 0);
  TORCH_CHECK(nb != 0, "admmq: cp workspace planning failed: ", admmq_last_error());
  at::Tensor ws = workspace(nb, keep[0]);
  check_rc(admmq_cp_rel_error(L.data(), n, out.data_ptr<double>(), ws.data_ptr(), ws.numel(), stream_of(keep[0])),
           "cp_rel_error");
  return out;
}

at::Tensor cp_rel_error_meta(at::TensorList W, at::TensorList factors) {
  return at::empty({static_cast<int64_t>(W.size())}, W[0].options().dtype(at::kDouble));
}

}  // namespace

TORCH_LIBRARY(admmq, m) {
  m.def("admm_iteration_batched(Tensor[] H, Tensor(a!)[] U, Tensor[] F, Tensor[] G, int max_iter, float eps, "
        "int bits, int qscheme, int num_attempts=200, bool check_spd=True, bool debug=False, int solve=-1, bool check_fault=True) "
        "-> (Tensor[] H_out, Tensor info, Tensor[] HT, Tensor[] X)");
  m.def("quantize_batched(Tensor[] x, int bits, int qscheme, int num_attempts=200, float? tmin=None, "
        "float? tmax=None) -> Tensor[]");
  m.def("quantize_channel(Tensor x, int bits, int qscheme, int dim) -> Tensor");
  m.def("cp_gram_mttkrp(Tensor[] W, Tensor[] factors, int mode) -> (Tensor[] G, Tensor[] F)");
  m.def("cp_rel_error(Tensor[] W, Tensor[] factors) -> Tensor");
  m.def("fault_repairs(bool reset=False) -> int", &fault_repairs);
}

TORCH_LIBRARY_IMPL(admmq, CUDA, m) {
  m.impl("admm_iteration_batched", &admm_batched_cuda);
  m.impl("quantize_batched", &quantize_batched_cuda);
  m.impl("quantize_channel", &quantize_channel_cuda);
  m.impl("cp_gram_mttkrp", &cp_gram_mttkrp_cuda);
  m.impl("cp_rel_error", &cp_rel_error_cuda);
}

TORCH_LIBRARY_IMPL(admmq, Meta, m) {
  m.impl("admm_iteration_batched", &admm_batched_meta);
  m.impl("quantize_batched", &quantize_batched_meta);
  m.impl("quantize_channel", &quantize_channel_meta);
  m.impl("cp_gram_mttkrp", &cp_gram_mttkrp_meta);
  m.impl("cp_rel_error", &cp_rel_error_meta);
}
