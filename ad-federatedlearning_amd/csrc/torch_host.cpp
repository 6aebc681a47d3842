// torch_host.cpp — the host-resident channel path's per-tensor torch plumbing, one call per batch
// (adfl_amd/Channel/quant.py). ADFL hands the channel CPU state dicts of ~256 tensors (Src/ADFL/model.py:195-197)
// and expects 256 owned tensors back from every on_client_send / on_server_receive (quant.py:74-112): their
// creation, and reading each payload's quantizer, cost ~2.5 us per tensor per Python call — about 0.6 ms per
// direction on C3, as much as the PCIe copies they overlap. Here each batch is one call into ATen:
//   empty_f32_like(like)            fresh contiguous fp32 tensors shaped like `like`, on each one's device (the
//                                   decode's outputs)
//   empty_qint8_like(like, scales)  per-tensor affine qint8 tensors, zero point 0, scale[k], on each like's
//                                   device (the payloads, as torch.quantize_per_tensor(x, scale, 0, qint8) makes them)
//   qint8_meta(q)                   for payload tensors: whether every one is a per-tensor affine qint8 tensor
//                                   with zero point 0, whether all are contiguous CPU tensors, their element
//                                   counts, fp32 scales (fbgemm uses q_scale() as fp32, quant.py:110) and
//                                   data pointers
//   data_ptrs(ts)                   the tensors' data pointers
//   payload_kinds(ts)               per payload 0: ndim <= 1 (passed through), 1: ndim > 1 and quantized (decoded),
//                                   2: ndim > 1 otherwise — _receive's three cases (quant.py:107-112)
//   variable_data(ts)               t.data for each (what _receive hands back for a passthrough entry)
//   tensor_meta(ts)                 per tensor: ndim, numel, whether fp32, whether a contiguous CPU tensor — what
//                                   _quantize_params and the staging choose by, for a whole state dict at once
//   host_bytes(ts, elem)            whether every tensor is a contiguous CPU tensor of elem-byte elements, their
//                                   element counts and data pointers (the stochastic channels' planes and inputs)
//   empty_like_dtype(like, code)    fresh contiguous tensors shaped like `like`, on each one's device, uint8 /
//                                   int8 / fp32 (code 0 / 1 / 2): the stochastic encode's level and sign planes
//   byte_planes(ts)                 whether every tensor is a contiguous CPU uint8 / int8 plane (the stochastic
//                                   codecs' levels, exponents and signs), their element counts and data pointers
//   empty_1d(numel, code)           fresh 1-D CPU tensors of the given element counts, uint8 / int8 / fp32 (the
//                                   packed int4 channel's payloads: ceil(n/2) bytes each)
//   device_ptrs(ts, index, elem)    whether every tensor is a contiguous tensor of elem-byte elements on cuda:index,
//                                   their element counts and data pointers (a device-resident dict's one-launch
//                                   gather / scatter)
//   shapes_equal(lists)             whether every list holds tensors of the first list's shapes, index by index
//                                   (receive_mean's K updates of one model)
//   entry_meta_k(lists)             for K lists of one model's entries: per entry, whether all K are contiguous
//                                   CPU tensors of one dtype and shape, its dtype (0 fp32, 1 int64, 2 other) and
//                                   element count (receive_mean's host aggregate of biases and statistics)
//   concat_rows(lists, idx)         [K, total]: row k = list k's entries idx concatenated (one copy each)
//   split_owned(flat, like)         owned tensors shaped like `like`, filled from consecutive pieces of flat
// Every returned pointer table is an int64 CPU tensor (the native copy pool's piece lists).
#include <torch/extension.h>

#include <algorithm>
#include <cstdint>
#include <cstring>
#include <tuple>
#include <vector>

namespace {

std::tuple<std::vector<at::Tensor>, at::Tensor> empty_f32_like(const std::vector<at::Tensor>& like) {
  std::vector<at::Tensor> out;
  out.reserve(like.size());
  at::Tensor ptrs = at::empty({(int64_t)like.size()}, at::kLong);
  int64_t* p = ptrs.data_ptr<int64_t>();
  const auto opts = at::TensorOptions().dtype(at::kFloat);
  for (size_t k = 0; k < like.size(); ++k) {
    out.push_back(at::empty(like[k].sizes(), opts.device(like[k].device())));
    p[k] = (int64_t)(intptr_t)out.back().data_ptr();
  }
  return {std::move(out), ptrs};
}

std::tuple<std::vector<at::Tensor>, at::Tensor> empty_qint8_like(const std::vector<at::Tensor>& like,
                                                                 const at::Tensor& scales) {
  TORCH_CHECK(scales.scalar_type() == at::kFloat && scales.is_contiguous() && !scales.is_cuda() &&
                  scales.numel() == (int64_t)like.size(),
              "empty_qint8_like: one fp32 CPU scale per tensor");
  const float* s = scales.data_ptr<float>();
  std::vector<at::Tensor> out;
  out.reserve(like.size());
  at::Tensor ptrs = at::empty({(int64_t)like.size()}, at::kLong);
  int64_t* p = ptrs.data_ptr<int64_t>();
  const auto opts = at::TensorOptions().dtype(at::kQInt8);
  for (size_t k = 0; k < like.size(); ++k) {
    out.push_back(at::_empty_affine_quantized(like[k].sizes(), opts.device(like[k].device()), (double)s[k], 0));
    p[k] = (int64_t)(intptr_t)out.back().data_ptr();
  }
  return {std::move(out), ptrs};
}

std::tuple<bool, bool, at::Tensor, at::Tensor, at::Tensor> qint8_meta(const std::vector<at::Tensor>& q) {
  const int64_t n = (int64_t)q.size();
  at::Tensor numel = at::empty({n}, at::kLong), scales = at::empty({n}, at::kFloat), ptrs = at::empty({n}, at::kLong);
  int64_t* ne = numel.data_ptr<int64_t>();
  float* sc = scales.data_ptr<float>();
  int64_t* pt = ptrs.data_ptr<int64_t>();
  bool ok = true, host = true;
  for (int64_t k = 0; k < n; ++k) {
    const at::Tensor& t = q[k];
    const bool quant = t.is_quantized() && t.scalar_type() == at::kQInt8 && t.qscheme() == at::kPerTensorAffine &&
                       t.q_zero_point() == 0;
    ok = ok && quant;
    host = host && !t.is_cuda() && t.is_contiguous();
    ne[k] = t.numel();
    sc[k] = quant ? (float)t.q_scale() : 0.0f;
    pt[k] = (int64_t)(intptr_t)t.data_ptr();
  }
  return {ok, host, numel, scales, ptrs};
}

at::Tensor data_ptrs(const std::vector<at::Tensor>& ts) {
  at::Tensor ptrs = at::empty({(int64_t)ts.size()}, at::kLong);
  int64_t* p = ptrs.data_ptr<int64_t>();
  for (size_t k = 0; k < ts.size(); ++k) p[k] = (int64_t)(intptr_t)ts[k].data_ptr();
  return ptrs;
}

at::Tensor payload_kinds(const std::vector<at::Tensor>& ts) {
  at::Tensor k = at::empty({(int64_t)ts.size()}, at::kByte);
  uint8_t* p = k.data_ptr<uint8_t>();
  for (size_t i = 0; i < ts.size(); ++i) p[i] = ts[i].dim() <= 1 ? 0 : (ts[i].is_quantized() ? 1 : 2);
  return k;
}

std::vector<at::Tensor> variable_data(const std::vector<at::Tensor>& ts) {
  std::vector<at::Tensor> out;
  out.reserve(ts.size());
  for (const auto& t : ts) out.push_back(t.variable_data());
  return out;
}

std::tuple<at::Tensor, at::Tensor, at::Tensor, at::Tensor> tensor_meta(const std::vector<at::Tensor>& ts) {
  const int64_t n = (int64_t)ts.size();
  at::Tensor ndim = at::empty({n}, at::kByte), numel = at::empty({n}, at::kLong), f32 = at::empty({n}, at::kBool),
             host = at::empty({n}, at::kBool);
  uint8_t* nd = ndim.data_ptr<uint8_t>();
  int64_t* ne = numel.data_ptr<int64_t>();
  bool* f = f32.data_ptr<bool>();
  bool* h = host.data_ptr<bool>();
  for (int64_t i = 0; i < n; ++i) {
    const at::Tensor& t = ts[i];
    nd[i] = (uint8_t)std::min<int64_t>(t.dim(), 255);
    ne[i] = t.numel();
    f[i] = t.scalar_type() == at::kFloat;
    h[i] = !t.is_cuda() && t.is_contiguous();
  }
  return {ndim, numel, f32, host};
}

std::tuple<bool, at::Tensor, at::Tensor> host_bytes(const std::vector<at::Tensor>& ts, int64_t elem) {
  const int64_t n = (int64_t)ts.size();
  at::Tensor numel = at::empty({n}, at::kLong), ptrs = at::empty({n}, at::kLong);
  int64_t* ne = numel.data_ptr<int64_t>();
  int64_t* pt = ptrs.data_ptr<int64_t>();
  bool ok = true;
  for (int64_t k = 0; k < n; ++k) {
    const at::Tensor& t = ts[k];
    ok = ok && !t.is_cuda() && t.is_contiguous() && (int64_t)t.element_size() == elem;
    ne[k] = t.numel();
    pt[k] = (int64_t)(intptr_t)t.data_ptr();
  }
  return {ok, numel, ptrs};
}

std::tuple<std::vector<at::Tensor>, at::Tensor> empty_like_dtype(const std::vector<at::Tensor>& like, int64_t code) {
  TORCH_CHECK(code >= 0 && code <= 2, "empty_like_dtype: code 0 (uint8), 1 (int8) or 2 (float32)");
  const at::ScalarType st = code == 0 ? at::kByte : (code == 1 ? at::kChar : at::kFloat);
  std::vector<at::Tensor> out;
  out.reserve(like.size());
  at::Tensor ptrs = at::empty({(int64_t)like.size()}, at::kLong);
  int64_t* p = ptrs.data_ptr<int64_t>();
  const auto opts = at::TensorOptions().dtype(st);
  for (size_t k = 0; k < like.size(); ++k) {
    out.push_back(at::empty(like[k].sizes(), opts.device(like[k].device())));
    p[k] = (int64_t)(intptr_t)out.back().data_ptr();
  }
  return {std::move(out), ptrs};
}

std::tuple<bool, at::Tensor, at::Tensor> byte_planes(const std::vector<at::Tensor>& ts) {
  const int64_t n = (int64_t)ts.size();
  at::Tensor numel = at::empty({n}, at::kLong), ptrs = at::empty({n}, at::kLong);
  int64_t* ne = numel.data_ptr<int64_t>();
  int64_t* pt = ptrs.data_ptr<int64_t>();
  bool ok = true;
  for (int64_t k = 0; k < n; ++k) {
    const at::Tensor& t = ts[k];
    ok = ok && !t.is_cuda() && t.is_contiguous() && t.element_size() == 1 && !t.is_quantized() &&
         !t.is_floating_point() && t.scalar_type() != at::kBool;
    ne[k] = t.numel();
    pt[k] = (int64_t)(intptr_t)t.data_ptr();
  }
  return {ok, numel, ptrs};
}

std::tuple<std::vector<at::Tensor>, at::Tensor> empty_1d(const at::Tensor& numel, int64_t code) {
  TORCH_CHECK(numel.scalar_type() == at::kLong && !numel.is_cuda() && numel.is_contiguous(), "empty_1d: int64 counts");
  TORCH_CHECK(code >= 0 && code <= 2, "empty_1d: code 0 (uint8), 1 (int8) or 2 (float32)");
  const at::ScalarType st = code == 0 ? at::kByte : (code == 1 ? at::kChar : at::kFloat);
  const int64_t n = numel.numel();
  const int64_t* ne = numel.data_ptr<int64_t>();
  std::vector<at::Tensor> out;
  out.reserve((size_t)n);
  at::Tensor ptrs = at::empty({n}, at::kLong);
  int64_t* p = ptrs.data_ptr<int64_t>();
  const auto opts = at::TensorOptions().dtype(st);
  for (int64_t k = 0; k < n; ++k) {
    out.push_back(at::empty({ne[k]}, opts));
    p[k] = (int64_t)(intptr_t)out.back().data_ptr();
  }
  return {std::move(out), ptrs};
}

std::tuple<bool, at::Tensor, at::Tensor> device_ptrs(const std::vector<at::Tensor>& ts, int64_t device_index,
                                                      int64_t elem) {
  const int64_t n = (int64_t)ts.size();
  at::Tensor numel = at::empty({n}, at::kLong), ptrs = at::empty({n}, at::kLong);
  int64_t* ne = numel.data_ptr<int64_t>();
  int64_t* p = ptrs.data_ptr<int64_t>();
  bool ok = true;
  for (int64_t k = 0; k < n; ++k) {
    const at::Tensor& t = ts[k];
    ok = ok && t.is_cuda() && t.device().index() == device_index && t.is_contiguous() &&
         (int64_t)t.element_size() == elem;
    ne[k] = t.numel();
    p[k] = (int64_t)(intptr_t)t.data_ptr();
  }
  return {ok, numel, ptrs};
}

bool shapes_equal(const std::vector<std::vector<at::Tensor>>& lists) {
  if (lists.empty()) return true;
  const auto& a = lists[0];
  for (size_t r = 1; r < lists.size(); ++r) {
    const auto& b = lists[r];
    if (b.size() != a.size()) return false;
    for (size_t k = 0; k < a.size(); ++k)
      if (!a[k].sizes().equals(b[k].sizes())) return false;
  }
  return true;
}

std::tuple<at::Tensor, at::Tensor, at::Tensor> entry_meta_k(const std::vector<std::vector<at::Tensor>>& lists) {
  TORCH_CHECK(!lists.empty(), "entry_meta_k: no lists");
  const size_t n = lists[0].size();
  for (const auto& l : lists) TORCH_CHECK(l.size() == n, "entry_meta_k: lists of different lengths");
  at::Tensor uni = at::empty({(int64_t)n}, at::kBool), code = at::empty({(int64_t)n}, at::kChar),
             numel = at::empty({(int64_t)n}, at::kLong);
  bool* u = uni.data_ptr<bool>();
  int8_t* c = code.data_ptr<int8_t>();
  int64_t* ne = numel.data_ptr<int64_t>();
  for (size_t i = 0; i < n; ++i) {
    const at::Tensor& t0 = lists[0][i];
    bool ok = !t0.is_cuda() && t0.is_contiguous();
    for (size_t r = 1; ok && r < lists.size(); ++r) {
      const at::Tensor& t = lists[r][i];
      ok = !t.is_cuda() && t.is_contiguous() && t.scalar_type() == t0.scalar_type() && t.sizes().equals(t0.sizes());
    }
    u[i] = ok;
    c[i] = t0.scalar_type() == at::kFloat ? 0 : (t0.scalar_type() == at::kLong ? 1 : 2);
    ne[i] = t0.numel();
  }
  return {uni, code, numel};
}

at::Tensor concat_rows(const std::vector<std::vector<at::Tensor>>& lists, const at::Tensor& idx) {
  TORCH_CHECK(!lists.empty() && idx.scalar_type() == at::kLong && idx.numel() > 0, "concat_rows: bad arguments");
  const int64_t* ix = idx.data_ptr<int64_t>();
  const int64_t m = idx.numel();
  const at::Tensor& first = lists[0][ix[0]];
  int64_t total = 0;
  for (int64_t j = 0; j < m; ++j) total += lists[0][ix[j]].numel();
  at::Tensor out = at::empty({(int64_t)lists.size(), total}, first.options());
  const int64_t es = (int64_t)first.element_size();
  for (size_t r = 0; r < lists.size(); ++r) {
    char* dst = static_cast<char*>(out[r].data_ptr());
    for (int64_t j = 0; j < m; ++j) {
      const at::Tensor& t = lists[r][ix[j]];
      TORCH_CHECK(!t.is_cuda() && t.is_contiguous() && t.scalar_type() == first.scalar_type(),
                  "concat_rows: entries must be contiguous CPU tensors of one dtype");
      const int64_t nb = t.numel() * es;
      std::memcpy(dst, t.data_ptr(), (size_t)nb);
      dst += nb;
    }
  }
  return out;
}

std::vector<at::Tensor> split_owned(const at::Tensor& flat, const std::vector<at::Tensor>& like) {
  TORCH_CHECK(!flat.is_cuda() && flat.is_contiguous(), "split_owned: a contiguous CPU tensor");
  std::vector<at::Tensor> out;
  out.reserve(like.size());
  const char* src = static_cast<const char*>(flat.data_ptr());
  const int64_t es = (int64_t)flat.element_size();
  int64_t off = 0;
  for (const auto& l : like) {
    at::Tensor t = at::empty(l.sizes(), flat.options());
    TORCH_CHECK(off + t.numel() <= flat.numel(), "split_owned: flat too short");
    std::memcpy(t.data_ptr(), src + off * es, (size_t)(t.numel() * es));
    off += t.numel();
    out.push_back(std::move(t));
  }
  return out;
}

}  // namespace

PYBIND11_MODULE(TORCH_EXTENSION_NAME, m) {
  m.def("empty_f32_like", &empty_f32_like);
  m.def("empty_qint8_like", &empty_qint8_like);
  m.def("qint8_meta", &qint8_meta);
  m.def("data_ptrs", &data_ptrs);
  m.def("payload_kinds", &payload_kinds);
  m.def("variable_data", &variable_data);
  m.def("tensor_meta", &tensor_meta);
  m.def("host_bytes", &host_bytes);
  m.def("empty_like_dtype", &empty_like_dtype);
  m.def("shapes_equal", &shapes_equal);
  m.def("device_ptrs", &device_ptrs);
  m.def("empty_1d", &empty_1d);
  m.def("byte_planes", &byte_planes);
  m.def("entry_meta_k", &entry_meta_k);
  m.def("concat_rows", &concat_rows);
  m.def("split_owned", &split_owned);
}
