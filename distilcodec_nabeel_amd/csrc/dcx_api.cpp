// Host runtime behind include/distilcodec_amd.h: checkpoint ingestion (weight-norm folding and
// kernel-layout packing), workspace planning and stage orchestration on one HIP stream.
//
// Stage call graphs follow the reference modules (paths under the reference checkout):
//   mel      mel_spec.py:26-57,100-122
//   encode   encoders.py:68-76, convnext_utils.py:186-282
//   vq       grfvq.py:105-146, residual_vq.py:103-259, vector_quantize_pytorch.py:41-45,462-538
//   generate generators.py:118-147, convnext_utils.py:106-113,137-138
#include <hip/hip_runtime.h>

#include <atomic>
#include <climits>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <string>
#include <vector>

#include "../../include/distilcodec_amd.h"
#include "dcx_kernels.h"

using dcx::ConvParams;

namespace {

struct HostTensor {
  std::vector<int64_t> shape;
  std::vector<float> data;
  int64_t numel() const {
    int64_t n = 1;
    for (auto s : shape) n *= s;
    return n;
  }
};

struct ConvW {
  float* w = nullptr;
  unsigned short* w6 = nullptr;  // bf16 3-plane split, x6 kernel layout
  unsigned short* wc = nullptr;  // 1x1 convs: hi plane only, [Cin/32][Cout][32] (bf16 mode, conv_gemm_bf16dm)
  unsigned short* w3 = nullptr;  // h3 arithmetic: fp16 h / l of w * 2^w3_shift (ConvParams::w3)
  int w3_shift = 0;
  float* b = nullptr;
  float* b16 = nullptr;  // the bias rounded to bf16 (bf16 mode: autocast casts it with the weight)
  int cin = 0, cout = 0, taps = 1, phases = 1, in_step = 1, out_mul = 1;
  int in_base[dcx::kMaxPhases] = {0};
  // h3 activation range (round 6, dcx_kernels.h h2_shift): |out| <= g_abs max|in| + b_abs, g_abs the
  // largest absolute row sum of the weights over (phase, output channel), b_abs = max |bias|
  float g_abs = 0.f, b_abs = 0.f;
};

struct LnW {
  float* w = nullptr;
  float* b = nullptr;
  int C = 0;
};

struct BlockW {  // ConvNeXtBlock
  int C = 0;
  float *dww = nullptr, *dwb = nullptr, *gamma = nullptr;
  LnW ln;
  ConvW pw1, pw2;
};

struct Err {
  int code;
  std::string msg;
};

struct ProfRec {
  int id;
  int ev0, ev1;
  double flops, bytes;
};

struct Bump {  // workspace carve-out, 256-byte aligned
  char* base;
  size_t cap, off = 0;
  bool dry;
  Bump(void* p, size_t c, bool d) : base((char*)p), cap(c), dry(d) {}
  float* f(size_t n) { return (float*)raw(n * sizeof(float)); }
  int* i(size_t n) { return (int*)raw(n * sizeof(int)); }
  unsigned short* u16(size_t n) { return (unsigned short*)raw(n * sizeof(unsigned short)); }
  void* raw(size_t bytes) {
    size_t o = (off + 255) & ~(size_t)255;
    off = o + bytes;
    return dry ? nullptr : base + o;
  }
  bool ok() const { return off <= cap; }
};

}  // namespace

struct dcx_codec {
  dcx_config cfg;
  int device = 0;
  std::string err;
  std::map<std::string, HostTensor> host;
  bool finalized = false, has_gen = false;
  std::vector<void*> allocs;

  ConvW dft, melfb;
  ConvW stem;
  LnW stem_ln, enc_norm;
  LnW ds_ln[4];
  ConvW ds_conv[4];
  std::vector<BlockW> blocks[4];

  ConvW vq_down, vq_pin, vq_up;
  BlockW vq_down_blk, vq_up_blk;
  int* rflag = nullptr;  // device RangeFlag bits (dcx_range_flags; round 6)
  float *codebook = nullptr, *e2 = nullptr, *ptable = nullptr;
  double* e2d = nullptr;          // |e|^2 per code in fp64 (the rescore)
  float emax = 0.f, e2max = 0.f;  // largest codebook row norm / squared norm (prefilter bound)
  float dmax = 0.f;               // largest |e - bf16(e)| over the codes (vq_prefilter_b1's bound)
  int* vq_stats = nullptr;        // [rows rescored, codes rescored] (dcx_vq_rescore_stats)
  bool vq_stats_on = false;       // counted from the first dcx_vq_rescore_stats call on
  unsigned short* codebook6 = nullptr;
  unsigned short* codebook_bk = nullptr;  // hi/mid per K32 step (vq_prefilter_bq / _dm; DCX_VQ_OLD builds)
  unsigned short* codebook_b1 = nullptr;  // [CD/32][NC][32] bf16 hi (vq_prefilter_b1)
  unsigned short* ptable6 = nullptr;  // decode table as activation planes (x6 mode gathers)
  // bf16-mode decode table (planes; mid = lo = 0): project_out under autocast, bf16(bf16(E) W16^T + b16)
  unsigned short* ptable6b = nullptr;
  int gemm_mode = DCX_GEMM_X6;
  // fused ResBlock pairs for the C = 32 / 64 generator stages (conv_res_pair); DCX_NO_RESPAIR=1 at
  // dcx_create keeps the per-conv launches (A/B comparisons)
  bool res_pair = true;
  // compact bf16 activations between bf16-mode producers and conv_gemm_bf16dm / vq_prefilter_bk;
  // DCX_NO_COMPACT=1 at dcx_create keeps the planes layout (A/B comparisons, same bits)
  bool compact = true;
  // rescore candidate-list capacity per searched row (VqScratch); DCX_VQ_PAIRS_PER_ROW at dcx_create
  // (0: every uncertified row is rescored in place, the overflow path; tests)
  int vq_pairs_per_row = 128;
  // split-K latency mode (dcx_set_split_k): at most split_k K-slices per few-tile x6 conv; the
  // partial sums live in the first kSplitScratch bytes of each stage call's workspace.  split_buf
  // points there only for the duration of one stage call (CallScope), which `busy` makes exclusive.
  int split_k = 0;
  float* split_buf = nullptr;
  // A/B and test switches, read from the environment once at dcx_create (knobs_from_env) and changed
  // only by dcx_set_knob; every launcher gets them through its parameters
  dcx::Knobs knobs;
  std::atomic<int> busy{0};
  // a second stream for the encoder's second half-batch (stage_encode), forked from and joined to
  // the caller's stream by events; created at dcx_finalize on the handle's device
  hipStream_t side = nullptr;
  hipEvent_t fork_ev = nullptr, join_ev = nullptr;
  bool no_fork = false;  // inside a whole-path half (stage_encode_decode): the encoder does not fork again

  ConvW conv_pre;
  ConvW ups[8];
  ConvW res[8][4][4][2];
  float* post_w = nullptr;
  float post_b = 0.f;

  bool prof = false;
  std::vector<hipEvent_t> events;
  int ev_used = 0;
  std::vector<ProfRec> pending;
  std::vector<std::string> prof_names;
  std::map<std::string, int> prof_ids;
  std::vector<int64_t> prof_launches;
  std::vector<double> prof_ms, prof_flops, prof_bytes;
};

namespace {

int fail(dcx_codec* h, int code, const std::string& m) {
  if (h) h->err = m;
  return code;
}

#define HIPCHK(h, expr)                                                                   \
  do {                                                                                    \
    hipError_t e_ = (expr);                                                               \
    if (e_ != hipSuccess)                                                                 \
      return fail(h, DCX_ERR_HIP, std::string(#expr) + ": " + hipGetErrorString(e_));     \
  } while (0)

#define RUN(expr)             \
  do {                        \
    int rc_ = (expr);         \
    if (rc_ != DCX_OK) return rc_; \
  } while (0)

// ----------------------------------------------------------------------------------------
// profiling
// ----------------------------------------------------------------------------------------
int prof_event(dcx_codec* h) {
  if (h->ev_used == (int)h->events.size()) {
    hipEvent_t e;
    if (hipEventCreate(&e) != hipSuccess) return -1;
    h->events.push_back(e);
  }
  return h->ev_used++;
}

struct ProfScope {
  dcx_codec* h;
  hipStream_t s;
  int e0 = -1;
  ProfScope(dcx_codec* h_, hipStream_t s_) : h(h_), s(s_) {
    if (h->prof) {
      e0 = prof_event(h);
      if (e0 >= 0) hipEventRecord(h->events[e0], s);
    }
  }
  void done(const char* name, double flops, double bytes) {
    if (!h->prof || e0 < 0) return;
    int e1 = prof_event(h);
    if (e1 < 0) return;
    hipEventRecord(h->events[e1], s);
    auto it = h->prof_ids.find(name);
    int id;
    if (it == h->prof_ids.end()) {
      id = (int)h->prof_names.size();
      h->prof_ids[name] = id;
      h->prof_names.push_back(name);
      h->prof_launches.push_back(0);
      h->prof_ms.push_back(0);
      h->prof_flops.push_back(0);
      h->prof_bytes.push_back(0);
    } else {
      id = it->second;
    }
    h->pending.push_back({id, e0, e1, flops, bytes});
  }
};

void prof_collect(dcx_codec* h) {
  if (h->pending.empty()) return;
  hipDeviceSynchronize();
  for (auto& r : h->pending) {
    float ms = 0.f;
    hipEventElapsedTime(&ms, h->events[r.ev0], h->events[r.ev1]);
    h->prof_launches[r.id] += 1;
    h->prof_ms[r.id] += ms;
    h->prof_flops[r.id] += r.flops;
    h->prof_bytes[r.id] += r.bytes;
  }
  h->pending.clear();
  h->ev_used = 0;
}

// ----------------------------------------------------------------------------------------
// weight ingestion
// ----------------------------------------------------------------------------------------
const HostTensor* find(dcx_codec* h, const std::string& k) {
  auto it = h->host.find(k);
  return it == h->host.end() ? nullptr : &it->second;
}

// Effective weight, folding weight norm (torch._weight_norm(v, g, dim=0)) in fp64.
bool get_weight(dcx_codec* h, const std::string& prefix, HostTensor& out) {
  if (auto t = find(h, prefix + ".weight")) {
    out = *t;
    return true;
  }
  const char* pairs[2][2] = {{".parametrizations.weight.original0", ".parametrizations.weight.original1"},
                             {".weight_g", ".weight_v"}};
  for (auto& pr : pairs) {
    auto g = find(h, prefix + pr[0]);
    auto v = find(h, prefix + pr[1]);
    if (g && v) {
      out.shape = v->shape;
      out.data.resize(v->data.size());
      const int64_t d0 = v->shape[0], inner = v->numel() / d0;
      if ((int64_t)g->data.size() != d0) return false;
      for (int64_t i = 0; i < d0; ++i) {
        double nrm = 0;
        for (int64_t j = 0; j < inner; ++j) nrm += (double)v->data[i * inner + j] * v->data[i * inner + j];
        nrm = std::sqrt(nrm);
        const double sc = (double)g->data[i] / nrm;
        for (int64_t j = 0; j < inner; ++j) out.data[i * inner + j] = (float)(sc * v->data[i * inner + j]);
      }
      return true;
    }
  }
  return false;
}

unsigned short bf16_rne(float x) {
  unsigned u;
  std::memcpy(&u, &x, 4);
  return (unsigned short)((u + 0x7FFFu + ((u >> 16) & 1u)) >> 16);
}
float bf16_f(unsigned short b) {
  unsigned u = (unsigned)b << 16;
  float f;
  std::memcpy(&f, &u, 4);
  return f;
}
// x = hi + mid + lo, the same split the x6 kernel applies to activations.
void split3_host(float x, unsigned short& h, unsigned short& m, unsigned short& l) {
  h = bf16_rne(x);
  const float r1 = x - bf16_f(h);
  m = bf16_rne(r1);
  const float r2 = r1 - bf16_f(m);
  l = bf16_rne(r2);
}

struct Builder {
  dcx_codec* h;
  bool dry;  // validate names and shapes only: no device allocation
  Err e{DCX_OK, ""};

  bool bad() const { return e.code != DCX_OK; }
  void set(int c, const std::string& m) {
    if (!bad()) e = {c, m};
  }

  void* upload_raw(const void* src, size_t bytes) {
    if (bad() || dry) return nullptr;
    void* p = nullptr;
    if (hipMalloc(&p, bytes + 16) != hipSuccess) {
      set(DCX_ERR_OOM, "hipMalloc failed while uploading weights");
      return nullptr;
    }
    h->allocs.push_back(p);
    if (hipMemcpy(p, src, bytes, hipMemcpyHostToDevice) != hipSuccess) {
      set(DCX_ERR_HIP, "hipMemcpy failed while uploading weights");
      return nullptr;
    }
    return p;
  }
  float* upload(const std::vector<float>& v) {
    if (bad() || dry) return nullptr;
    void* p = nullptr;
    if (hipMalloc(&p, v.size() * sizeof(float) + 16) != hipSuccess) {
      set(DCX_ERR_OOM, "hipMalloc failed while uploading weights");
      return nullptr;
    }
    h->allocs.push_back(p);
    if (hipMemcpy(p, v.data(), v.size() * sizeof(float), hipMemcpyHostToDevice) != hipSuccess) {
      set(DCX_ERR_HIP, "hipMemcpy failed while uploading weights");
      return nullptr;
    }
    return (float*)p;
  }
  unsigned short* upload16(const std::vector<unsigned short>& v) {
    if (bad() || dry) return nullptr;
    void* p = nullptr;
    if (hipMalloc(&p, v.size() * sizeof(unsigned short) + 16) != hipSuccess) {
      set(DCX_ERR_OOM, "hipMalloc failed while uploading split weights");
      return nullptr;
    }
    h->allocs.push_back(p);
    if (hipMemcpy(p, v.data(), v.size() * sizeof(unsigned short), hipMemcpyHostToDevice) != hipSuccess) {
      set(DCX_ERR_HIP, "hipMemcpy failed while uploading split weights");
      return nullptr;
    }
    return (unsigned short*)p;
  }
  // fp32 packed [phases][cout][taps][cin] -> x6 layout [phase][tap][cin/16][cout][2][3][8] bf16
  unsigned short* split_pack(const std::vector<float>& pk, int phases, int cout, int taps, int cin) {
    if (bad() || dry) return nullptr;
    const int nch = cin / 16;
    std::vector<unsigned short> out((size_t)phases * taps * nch * cout * 48);
    for (int r = 0; r < phases; ++r)
      for (int m = 0; m < taps; ++m)
        for (int c = 0; c < nch; ++c)
          for (int o = 0; o < cout; ++o) {
            unsigned short* dst = &out[((((size_t)r * taps + m) * nch + c) * cout + o) * 48];
            const float* src = &pk[(((size_t)r * cout + o) * taps + m) * cin + c * 16];
            for (int hh = 0; hh < 2; ++hh)
              for (int j = 0; j < 8; ++j) {
                unsigned short a, b2, c2;
                split3_host(src[hh * 8 + j], a, b2, c2);
                dst[hh * 24 + 0 + j] = a;
                dst[hh * 24 + 8 + j] = b2;
                dst[hh * 24 + 16 + j] = c2;
              }
          }
    return upload16(out);
  }
  // fp32 packed [phases][cout][taps][cin] -> h3 layout [phase][tap][cin/32][cout][4 groups][h 8 | l 8]
  // fp16 of w * 2^shift, shift putting the largest |w| in [2^14, 2^15) (conv_gemm_x3dq / x3dw)
  unsigned short* h2_pack(const std::vector<float>& pk, int phases, int cout, int taps, int cin, int& shift) {
    if (bad() || dry) return nullptr;
    float mx = 0.f;
    for (float v : pk) mx = std::max(mx, std::fabs(v));
    int e = 0;
    if (mx > 0.f) std::frexp(mx, &e);  // mx = f * 2^e, f in [0.5, 1)
    shift = mx > 0.f ? 15 - e : 0;
    const int nch = cin / 32;
    std::vector<unsigned short> out((size_t)phases * taps * nch * cout * 64);
    for (int r = 0; r < phases; ++r)
    for (int m = 0; m < taps; ++m)
      for (int c = 0; c < nch; ++c)
        for (int o = 0; o < cout; ++o) {
          unsigned short* dst = &out[((((size_t)r * taps + m) * nch + c) * cout + o) * 64];
          const float* src = &pk[(((size_t)r * cout + o) * taps + m) * cin + c * 32];
          for (int j = 0; j < 32; ++j) {
            const float x = std::ldexp(src[j], shift);
            const _Float16 hh = (_Float16)x;
            const _Float16 ll = (_Float16)(x - (float)hh);
            dst[(j >> 3) * 16 + (j & 7)] = __builtin_bit_cast(unsigned short, hh);
            dst[(j >> 3) * 16 + 8 + (j & 7)] = __builtin_bit_cast(unsigned short, ll);
          }
        }
    return upload16(out);
  }
  // fp32 packed [cout][cin] (one tap, one phase) -> [cin/32][cout][32] bf16 hi (conv_gemm_bf16dm)
  unsigned short* compact_pack(const std::vector<float>& pk, int cout, int cin) {
    if (bad() || dry) return nullptr;
    std::vector<unsigned short> out((size_t)cout * cin);
    for (int st = 0; st < cin / 32; ++st)
      for (int o = 0; o < cout; ++o)
        for (int j = 0; j < 32; ++j) out[((size_t)st * cout + o) * 32 + j] = bf16_rne(pk[(size_t)o * cin + st * 32 + j]);
    return upload16(out);
  }
  float* alloc(size_t n) {
    if (bad() || dry) return nullptr;
    void* p = nullptr;
    if (hipMalloc(&p, n * sizeof(float) + 16) != hipSuccess) {
      set(DCX_ERR_OOM, "hipMalloc failed");
      return nullptr;
    }
    h->allocs.push_back(p);
    return (float*)p;
  }

  const HostTensor* need(const std::string& k, std::vector<int64_t> shape) {
    auto t = find(h, k);
    if (!t) {
      set(DCX_ERR_MISSING_WEIGHT, "missing checkpoint tensor '" + k + "'");
      return nullptr;
    }
    if (t->numel() != [&] { int64_t n = 1; for (auto s : shape) n *= s; return n; }()) {
      set(DCX_ERR_INVALID_ARG, "checkpoint tensor '" + k + "' has the wrong number of elements");
      return nullptr;
    }
    return t;
  }
  float* vec(const std::string& k, int64_t n) {
    auto t = need(k, {n});
    return t ? upload(t->data) : nullptr;
  }
  // the same vector rounded to bf16 values (fp32 storage)
  float* vec_bf16(const std::string& k, int64_t n) {
    auto t = need(k, {n});
    if (!t) return nullptr;
    std::vector<float> r(t->data.size());
    for (size_t i = 0; i < r.size(); ++i) r[i] = bf16_f(bf16_rne(t->data[i]));
    return upload(r);
  }
  HostTensor weight(const std::string& prefix, std::vector<int64_t> shape) {
    HostTensor w;
    if (bad()) return w;
    if (!get_weight(h, prefix, w)) {
      set(DCX_ERR_MISSING_WEIGHT, "missing checkpoint weight '" + prefix + "'");
      return w;
    }
    int64_t n = 1;
    for (auto s : shape) n *= s;
    if (w.numel() != n) set(DCX_ERR_INVALID_ARG, "checkpoint weight '" + prefix + "' has the wrong shape");
    return w;
  }

  // h3 range bounds of a conv (ConvW::g_abs, b_abs) from its packed fp32 weights [phases][cout][kk]
  // and its bias
  static float round_up(double v) {
    float f = (float)v;
    if ((double)f < v) f = std::nextafter(f, INFINITY);
    return f;
  }
  void range_of(ConvW& c, const std::vector<float>& pk, int phases, int cout, size_t kk, const std::string& bias) {
    if (dry) return;
    double g = 0;
    for (int r = 0; r < phases; ++r)
      for (int o = 0; o < cout; ++o) {
        double sacc = 0;
        const float* row = &pk[((size_t)r * cout + o) * kk];
        for (size_t j = 0; j < kk; ++j) sacc += std::fabs((double)row[j]);
        g = std::max(g, sacc);
      }
    c.g_abs = round_up(g);
    double bm = 0;
    if (const HostTensor* t = bias.empty() ? nullptr : find(h, bias))
      for (float v : t->data) bm = std::max(bm, std::fabs((double)v));
    c.b_abs = round_up(bm);
  }

  // Conv1d / Linear weight [Cout][Cin][k] -> packed [Cout][k][Cin].
  // h3: also the h3 weights (conv_gemm_x3dq; the generator's ResBlock convs of the wide stages)
  ConvW conv(const std::string& prefix, int cin, int cout, int k, int dil, int pad, bool has_bias = true,
             bool h3 = false) {
    ConvW c;
    c.cin = cin; c.cout = cout; c.taps = k; c.in_step = dil; c.in_base[0] = -pad;
    HostTensor w = weight(prefix, {cout, cin, k});
    if (bad()) return c;
    std::vector<float> pk((size_t)cout * k * cin);
    for (int o = 0; o < cout; ++o)
      for (int i = 0; i < cin; ++i)
        for (int j = 0; j < k; ++j) pk[((size_t)o * k + j) * cin + i] = w.data[((size_t)o * cin + i) * k + j];
    c.w = upload(pk);
    if (cin % 16 == 0) c.w6 = split_pack(pk, 1, cout, k, cin);
    if (k == 1 && cin % 32 == 0) c.wc = compact_pack(pk, cout, cin);
    if (h3 && cin % 32 == 0) c.w3 = h2_pack(pk, 1, cout, k, cin, c.w3_shift);
    if (has_bias) {
      c.b = vec(prefix + ".bias", cout);
      c.b16 = vec_bf16(prefix + ".bias", cout);
    }
    range_of(c, pk, 1, cout, (size_t)k * cin, has_bias ? prefix + ".bias" : "");
    return c;
  }

  // ConvTranspose1d weight [Cin][Cout][k], stride s, padding (k-s)/2 -> s polyphase convs:
  // output o = q*s + r reads input q + base_r - m with tap j = (r+p)%s + m*s, m < k/s.
  ConvW convT(const std::string& prefix, int cin, int cout, int k, int s, bool h3 = false) {
    ConvW c;
    const int p = (k - s) / 2, taps = k / s;
    c.cin = cin; c.cout = cout; c.taps = taps; c.phases = s; c.in_step = -1; c.out_mul = s;
    HostTensor w = weight(prefix, {cin, cout, k});
    if (bad()) return c;
    std::vector<float> pk((size_t)s * cout * taps * cin);
    for (int r = 0; r < s; ++r) {
      const int jr = (r + p) % s;
      c.in_base[r] = (r + p - jr) / s;
      for (int o = 0; o < cout; ++o)
        for (int m = 0; m < taps; ++m)
          for (int i = 0; i < cin; ++i)
            pk[(((size_t)r * cout + o) * taps + m) * cin + i] = w.data[((size_t)i * cout + o) * k + jr + m * s];
    }
    c.w = upload(pk);
    if (cin % 16 == 0) c.w6 = split_pack(pk, s, cout, taps, cin);
    if (h3 && cin % 32 == 0) c.w3 = h2_pack(pk, s, cout, taps, cin, c.w3_shift);
    c.b = vec(prefix + ".bias", cout);
    c.b16 = vec_bf16(prefix + ".bias", cout);
    range_of(c, pk, s, cout, (size_t)taps * cin, prefix + ".bias");
    return c;
  }

  LnW ln(const std::string& prefix, int C) {
    LnW l;
    l.C = C;
    l.w = vec(prefix + ".weight", C);
    l.b = vec(prefix + ".bias", C);
    return l;
  }

  BlockW block(const std::string& p, int C) {
    BlockW b;
    b.C = C;
    auto dw = need(p + ".dwconv.weight", {C, 1, 7});
    if (dw) {
      std::vector<float> pk((size_t)7 * C);
      for (int c = 0; c < C; ++c)
        for (int j = 0; j < 7; ++j) pk[(size_t)j * C + c] = dw->data[(size_t)c * 7 + j];
      b.dww = upload(pk);
    }
    b.dwb = vec(p + ".dwconv.bias", C);
    b.ln = ln(p + ".norm", C);
    b.pw1 = conv(p + ".pwconv1", C, 4 * C, 1, 1, 0, true, true);
    b.pw2 = conv(p + ".pwconv2", 4 * C, C, 1, 1, 0, true, true);
    b.gamma = vec(p + ".gamma", C);
    return b;
  }
};

// Slaney mel filterbank (torchaudio melscale_fbanks norm='slaney', mel_scale='slaney').
double hz_to_mel(double f) {
  const double f_sp = 200.0 / 3, min_log_hz = 1000.0, min_log_mel = min_log_hz / f_sp, logstep = std::log(6.4) / 27.0;
  return f >= min_log_hz ? min_log_mel + std::log(f / min_log_hz) / logstep : f / f_sp;
}
double mel_to_hz(double m) {
  const double f_sp = 200.0 / 3, min_log_hz = 1000.0, min_log_mel = min_log_hz / f_sp, logstep = std::log(6.4) / 27.0;
  return m >= min_log_mel ? min_log_hz * std::exp(logstep * (m - min_log_mel)) : f_sp * m;
}
std::vector<double> mel_fb(int n_freqs, double fmin, double fmax, int n_mels, int sr) {
  std::vector<double> fb((size_t)n_freqs * n_mels, 0.0);
  std::vector<double> f_pts(n_mels + 2);
  const double m0 = hz_to_mel(fmin), m1 = hz_to_mel(fmax);
  for (int i = 0; i < n_mels + 2; ++i) f_pts[i] = mel_to_hz(m0 + (m1 - m0) * i / (n_mels + 1));
  for (int k = 0; k < n_freqs; ++k) {
    const double f = (double)(sr / 2) * k / (n_freqs - 1);
    for (int m = 0; m < n_mels; ++m) {
      const double down = (f - f_pts[m]) / (f_pts[m + 1] - f_pts[m]);
      const double up = (f_pts[m + 2] - f) / (f_pts[m + 2] - f_pts[m + 1]);
      double v = std::max(0.0, std::min(down, up));
      v *= 2.0 / (f_pts[m + 2] - f_pts[m]);
      fb[(size_t)k * n_mels + m] = v;
    }
  }
  return fb;
}

int64_t frames_of(const dcx_config& c, int64_t n) {
  const int64_t pad = (c.win - c.hop) / 2, padr = (c.win - c.hop + 1) / 2;
  const int64_t len = n + pad + padr;
  if (len < c.n_fft) return 0;
  return (len - c.n_fft) / c.hop + 1;
}

int max_gen_width(const dcx_config& c) {  // max over generator layers of channels x (L / T)
  int best = c.gen_channels, ch = c.gen_channels, up = 1;
  for (int i = 0; i < c.n_ups; ++i) {
    ch /= 2;
    up *= c.up_rates[i];
    best = std::max(best, ch * up);
  }
  return best;
}

// ----------------------------------------------------------------------------------------
// launches
// ----------------------------------------------------------------------------------------
// An activation tensor [rows][C]: fp32 and/or x6 planes ([rows][C/8][3][8] bf16, dcx_planes.h).
// c1: p holds the compact bf16 layout ([rows][C] hi only; bf16 mode, consumers conv_gemm_bf16dm /
// vq_prefilter_bk) instead of planes.
// h2: p holds the fp16 "h2" layout ([rows][C/32][8][8] h and l; the h3 generator arithmetic,
// consumer conv_gemm_x3dq).
// Range of a tensor (round 6, dcx_kernels.h h2_shift): in the h2 layout it holds x * 2^ash[clip]
// (ash null: ash_c for every clip); |x| <= max(amax[clip], amax_f) (amax null: amax_f), the input
// term of its consumers' bound programs.
// ash_row (one-tap consumers): a shift per row instead.
struct Rng {
  const int* ash = nullptr;
  int ash_c = 0;
  const float* amax = nullptr;
  float amax_f = 0.f;
  const int* ash_row = nullptr;
};
struct Act {
  float* f = nullptr;
  unsigned short* p = nullptr;
  bool c1 = false;
  bool h2 = false;
  Rng r;
  // per-row range buffers an h2 producer fills for a one-tap consumer (round 6): the shift and (for
  // LayerNorm outputs) the max |.| of each row
  int* row_ash = nullptr;
  float* row_amax = nullptr;
};
struct CAct {
  const float* f = nullptr;
  const unsigned short* p = nullptr;
  bool c1 = false;
  bool h2 = false;
  Rng r;
  CAct() = default;
  CAct(const float* f_, const unsigned short* p_, bool c1_ = false) : f(f_), p(p_), c1(c1_) {}
  CAct(const Act& a) : f(a.f), p(a.p), c1(a.c1), h2(a.h2), r(a.r) {}
};
// bound programs (dcx::RangeProg): c + sum of g * max(measured, floor) terms
void prog_add(dcx::RangeProg& p, float g, const Rng& r) {
  p.m[p.n] = r.amax;
  p.g[p.n] = g;
  p.f[p.n] = r.amax_f;
  ++p.n;
}
// |conv(x) + bias| <= g_abs max|x| + b_abs (|silu(v)|, |gelu(v)| <= |v|)
dcx::RangeProg prog_conv(const ConvW& w, const Rng& in) {
  dcx::RangeProg p{};
  p.c = w.b_abs;
  prog_add(p, w.g_abs, in);
  return p;
}
// per-row bound of a one-tap conv's output from its input rows' maxima (rowwise program)
dcx::RangeProg prog_conv_rows(const ConvW& w, const float* in_row_amax) {
  dcx::RangeProg p{};
  p.rowwise = 1;
  p.c = w.b_abs;
  p.m[0] = in_row_amax;
  p.g[0] = w.g_abs;
  p.n = 1;
  return p;
}

// planes layout for every GEMM operand (x6 and bf16 modes)
bool x6_mode(const dcx_codec* h) { return h->gemm_mode != DCX_GEMM_F32; }

// Workspace for a tensor consumed only by convs: planes in x6 mode, fp32 otherwise.
Act conv_input(dcx_codec* h, Bump& ws, size_t n) {
  Act a;
  if (x6_mode(h)) a.p = ws.u16(3 * n);
  else a.f = ws.f(n);
  return a;
}

struct ConvCall {
  CAct x;
  long long x_bstride;
  int batch, Lin, Lq, ldx;
  float* y = nullptr;            // v
  float* y2 = nullptr;           // silu(v), fp32
  unsigned short* y6 = nullptr;  // planes of v
  unsigned short* y6s = nullptr; // planes of silu(v)
  bool y6s_h2 = false;           // y6s in the h2 layout
  int y6c = 0;                   // y6 layout (ConvParams::y_compact): 0 planes, 1 compact bf16, 2 hm, 3 h2
  float* macc = nullptr;
  const float* res = nullptr;
  const float* gamma = nullptr;
  int epi = dcx::EPI_BIAS, mean = dcx::MEAN_NONE;
  bool exact = false;  // keep x6 arithmetic in bf16 mode (the reference's fp32 mel front end)
  bool silu_in = false;  // fp32 input: the conv consumes silu(x) (applied while staging)
  // h3 range (round 6): the bound program of an h2 output, where its per-clip shift goes, and where
  // the per-clip max |v| of the output goes (ConvParams::yb / y_ash / y_amax)
  dcx::RangeProg yb{};
  int* y_ash = nullptr;
  float* y_amax = nullptr;
  void silu_to(const Act& a) {
    y2 = a.f;
    y6s = a.p;
    y6s_h2 = a.h2;
  }
  void out_to(const Act& a) { y = a.f; y6 = a.p; y6c = a.c1 ? 1 : a.h2 ? 3 : 0; }
};

// Per-call range slots of the generator (round 6): measured per-clip maxima and h2 shifts, [slot][clip],
// zeroed once at the start of the call (one memset; capture-safe).
struct RangeArena {
  float* base = nullptr;
  int batch = 0, used = 0;
  static constexpr int kSlots = 320;
  void reserve(Bump& ws, int b) {
    batch = b;
    base = ws.f((size_t)kSlots * b);
  }
  // h3 range slots are only consumed by h2 tensors; a call past the capacity fails loudly
  float* amax() { return used < kSlots && base ? base + (size_t)(used++) * batch : nullptr; }
  int* ash() { return reinterpret_cast<int*>(amax()); }
  bool ok() const { return used < kSlots; }
};

// Planes-mode convs with Cout <= 64, Cin <= 128 and a tap halo take an fp32 input (split while
// staging; conv_gemm_x6w8 AF32).
bool f32_input_ok(const ConvW& w) { return w.cin <= 128 && w.cout <= 64 && w.taps >= 2; }

// ---- A/B and test switches (dcx::Knobs): names are the environment variables dcx_create reads ----
int* knob_slot(dcx::Knobs& k, const std::string& n) {
  if (n == "DCX_RP_R") return &k.rp_rows;
  if (n == "DCX_RP_OLD") return &k.rp_old;
  if (n == "DCX_RP_G64") return &k.rp_g64;
  if (n == "DCX_RP_SYNC") return &k.rp_sync;
  if (n == "DCX_RP_W4") return &k.rp_w4;
  if (n == "DCX_GELU_LUT") return &k.gelu_lut;
  if (n == "DCX_BF16_PERSIST") return &k.bf16_persist;
  if (n == "DCX_BF16_REG_EPI") return &k.bf16_reg_epi;
  if (n == "DCX_DWCONV_TILED") return &k.dwconv_tiled;
  if (n == "DCX_SPLIT_MIN_STEPS") return &k.split_min_steps;
  if (n == "DCX_SPLIT_GROUP_OFF") return &k.split_group_off;
  if (n == "DCX_H3") return &k.h3;
  if (n == "DCX_H3_BN") return &k.h3_bn;
  if (n == "DCX_H3_1X1") return &k.h3_1x1;
  if (n == "DCX_H3_SPLIT") return &k.h3_split;
  if (n == "DCX_H3_PAIRS") return &k.h3_pairs;
  if (n == "DCX_RP_RING") return &k.rp_ring;
  if (n == "DCX_ENC_STREAMS") return &k.enc_streams;
  return nullptr;
}

void knobs_from_env(dcx::Knobs& k) {
  static const char* const names[] = {"DCX_RP_R",         "DCX_RP_OLD",       "DCX_RP_G64",       "DCX_RP_SYNC",
                                      "DCX_RP_W4",        "DCX_GELU_LUT",     "DCX_BF16_PERSIST", "DCX_BF16_REG_EPI",
                                      "DCX_DWCONV_TILED", "DCX_SPLIT_MIN_STEPS", "DCX_SPLIT_GROUP_OFF",
                                      "DCX_H3",           "DCX_H3_BN",        "DCX_H3_1X1",
                                      "DCX_H3_SPLIT",     "DCX_H3_PAIRS",     "DCX_RP_RING",
                                      "DCX_ENC_STREAMS"};
  for (const char* n : names) {
    const char* e = std::getenv(n);
    if (e && *e) *knob_slot(k, n) = std::atoi(e);
  }
}

int conv_params(dcx_codec* h, const ConvW& w, const ConvCall& c, bool force_f32, ConvParams& p) {
  const bool x6 = x6_mode(h) && !force_f32;
  const bool x6_f32in = x6 && !c.x.p && c.x.f && f32_input_ok(w);
  if (c.silu_in && !x6_f32in) return fail(h, DCX_ERR_STATE, "internal: silu_in needs an fp32-input conv");
  if (x6 ? ((!c.x.p && !x6_f32in) || !w.w6) : !c.x.f)
    return fail(h, DCX_ERR_STATE, "internal: conv input missing for GEMM mode");
  p = ConvParams{};
  p.x = c.x.f;
  p.x6 = x6 ? c.x.p : nullptr;
  p.w = w.w;
  p.w6 = x6 ? w.w6 : nullptr;
  const bool one = x6 && h->gemm_mode == DCX_GEMM_BF16 && !c.exact;
  p.bias = one && w.b16 ? w.b16 : w.b;  // autocast rounds the bias with the other operands
  p.gamma = c.gamma;
  p.res = c.res;
  p.y = c.y;
  p.y2 = c.y2;
  p.y6 = c.y6;
  p.y6s = c.y6s;
  p.macc = c.macc;
  p.x_bstride = c.x_bstride;
  p.ldy = w.cout;
  p.y_bstride = (long long)c.Lq * w.out_mul * p.ldy;
  p.w_phase_stride = (long long)w.cout * w.taps * w.cin;
  p.Lin = c.Lin;
  p.Lq = c.Lq;
  p.Cin = w.cin;
  p.Cout = w.cout;
  p.ldx = c.ldx ? c.ldx : w.cin;
  p.taps = w.taps;
  p.in_step = w.in_step;
  p.out_mul = w.out_mul;
  for (int i = 0; i < dcx::kMaxPhases; ++i) p.in_base[i] = w.in_base[i];
  p.epi = c.epi;
  p.mean_mode = c.mean;
  p.nprod = one ? 1 : 6;
  p.round_bf16 = one;
  p.silu_in = c.silu_in;
  p.x_compact = x6 && c.x.p && c.x.c1 ? 1 : 0;
  p.y_compact = c.y6 ? c.y6c : 0;
  p.y6s_h2 = c.y6s && c.y6s_h2 ? 1 : 0;
  if (x6 && c.x.p && c.x.h2) {  // h3 arithmetic (conv_gemm_x3dq)
    if (!w.w3 || one) return fail(h, DCX_ERR_STATE, "internal: h2 input without h3 weights");
    p.x_compact = 3;
    p.w3 = w.w3;
    p.w3_shift = w.w3_shift;
    p.x_ash = c.x.r.ash;
    p.x_ash_c = c.x.r.ash_c;
    p.x_ash_row = c.x.r.ash_row;
    if (p.x_ash_row && (w.taps != 1 || w.phases != 1 || w.in_base[0] != 0))
      return fail(h, DCX_ERR_STATE, "internal: per-row input ranges need a one-tap conv");
  }
  p.y_ash = c.y_ash;
  p.y_amax = c.y_amax;
  p.yb = c.yb;
  p.rflag = h->rflag;
  p.wc = one && h->compact ? w.wc : nullptr;
  p.kn = &h->knobs;
  // compact inputs only feed one-product GEMMs; a compact output (the RNE hi value) may also be written
  // in x6 mode (x_pjt_in for vq_prefilter_b1)
  if (p.x_compact == 1 && !one) return fail(h, DCX_ERR_STATE, "internal: compact layout outside bf16 mode");
  if (p.y_compact == 2 && (!x6 || one)) return fail(h, DCX_ERR_STATE, "internal: hm layout outside x6 mode");
  if (p.y_compact == 3 && (!x6 || one)) return fail(h, DCX_ERR_STATE, "internal: h2 layout outside x6 mode");
  return DCX_OK;
}

// Whether a one-tap conv over `rows` rows runs on conv_gemm_bf16dm in this handle's mode, so its
// producer may write the compact bf16 layout (2 bytes per element instead of 6).
bool takes_compact(const dcx_codec* h, const ConvW& w, long long rows) {
  return h->compact && h->gemm_mode == DCX_GEMM_BF16 && w.wc && w.taps == 1 && w.phases == 1 && w.in_base[0] == 0 &&
         rows < (1LL << 31) && dcx::bf16dm_takes(w.cin, w.cout, (int)rows, w.cin, 1);
}

// Whether a generator conv with a tap halo (conv_pre, the ConvTs with Cout % 128 == 0) runs in h3
// arithmetic (conv_gemm_x3dw; Knobs::h3, x6 mode, not in the split-K latency mode), so its producer
// writes h2.
// The h3 tap kernels address a clip's input through one buffer descriptor: (rows + 1024) * Cin * 4
// bytes must stay under 2^31 (dcx_conv.hip x3dq_ok); longer clips (> ~11 min at the C = 256 stage)
// keep the x6 kernels, whose tiles rebase their descriptors.
bool h3_rows_ok(long long rows, int cin) { return (rows + 1024) * cin * 4LL < (1LL << 31); }

// rows: the conv's input rows per clip
bool takes_h3_conv(const dcx_codec* h, const ConvW& w, long long rows) {
  return h->knobs.h3 && h->gemm_mode == DCX_GEMM_X6 && h->split_k < 2 && w.w3 && w.taps >= 2 && w.cout % 128 == 0 &&
         h3_rows_ok(rows, w.cin);
}

// Whether a one-tap conv runs in h3 arithmetic (conv_gemm_x3dm; Knobs::h3_1x1, x6 mode, not in the
// split-K latency mode), so its producer writes the h2 layout.
bool takes_h3(const dcx_codec* h, const ConvW& w) {
  return h->knobs.h3_1x1 && h->gemm_mode == DCX_GEMM_X6 && h->split_k < 2 && w.w3 && w.taps == 1 && w.phases == 1 &&
         w.in_base[0] == 0 && w.cout % 128 == 0;
}

// algorithmic FLOPs and bytes of one conv (profiling)
double conv_flops(const ConvW& w, const ConvCall& c) { return 2.0 * c.batch * c.Lq * w.phases * w.cout * w.cin * w.taps; }
double conv_bytes(const ConvW& w, const ConvCall& c) {
  const double outs = (double)c.batch * c.Lq * w.phases * w.cout;
  return 4.0 * ((double)c.batch * c.Lin * w.cin + outs + (double)w.phases * w.cout * w.taps * w.cin);
}

// ---- split-K latency mode --------------------------------------------------------------------
// A conv whose output fits kSplitMaxOut floats and whose tiles leave most CUs idle (the few-tile
// kernels) runs as S K-slices over input-channel chunks, each writing fp32 partial sums, and one
// reduce kernel that sums them in slice order and applies the conv's epilogue.  Summation order
// (and so the low bits) then depends on S, i.e. on the tile count: the mode is opt-in and a clip
// alone is not bit-equal to the same clip in a batch.
constexpr long long kSplitMaxOut = 1LL << 21;        // floats per partial output (8 MiB)
constexpr int kSplitMax = 16;
constexpr size_t kSplitScratch = (size_t)kSplitMax * kSplitMaxOut * sizeof(float);

int split_factor(const dcx_codec* h, const ConvW& w, const ConvCall& c, const ConvParams& p) {
  if (h->split_k < 2 || !h->split_buf || p.nprod != 6 || !p.w6 || !p.x6 || p.x_compact || w.cout % 128) return 1;
  const long long out = (long long)c.batch * c.Lq * w.out_mul * w.cout;
  if (out > kSplitMaxOut || (w.cin / 16) % (w.taps % 2 ? 2 : 1)) return 1;
  // tiles of the 256 x 128 kernels the slices run on (conv_gemm_x6pp / x6lm, whatever the big-tile
  // rule would pick unsplit: in this mode the bits depend on the split anyway)
  const long long tiles = (long long)c.batch * ((c.Lq + 255) / 256) * std::max(1, w.cout / 128) * w.phases;
  if (tiles >= 128) return 1;
  // Knobs::split_min_steps (DCX_SPLIT_MIN_STEPS; A/B): convs with fewer K steps (taps x 16-channel
  // chunks) run unsplit
  if ((long long)w.taps * (w.cin / 16) < h->knobs.split_min_steps) return 1;
  const int unit = w.taps % 2 ? 2 : 1;  // chunks per slice: an even number of steps per slice
  const long long nunits = (w.cin / 16) / unit;
  return (int)std::min<long long>({(long long)std::min(h->split_k, kSplitMax), std::max<long long>(1, 256 / tiles), nunits});
}

int run_conv_split(dcx_codec* h, const ConvW& w, const ConvCall& c, const ConvParams& p, int S, hipStream_t s) {
  ProfScope ps(h, s);
  // one launch: slice sl of clip b is virtual clip sl * batch + b, its partial sums at that clip's
  // place in split_buf; then one reduce launch applies the epilogue
  ConvParams q = p;
  q.ksplit = S;
  q.kunit = w.taps % 2 ? 2 : 1;
  q.bias = q.gamma = q.res = nullptr;
  q.macc = nullptr;
  q.y = h->split_buf;
  q.y2 = nullptr;
  q.y6 = q.y6s = nullptr;
  q.epi = dcx::EPI_BIAS;
  q.mean_mode = dcx::MEAN_NONE;
  q.y_compact = 0;
  q.round_bf16 = 0;
  q.y_ash = nullptr;  // the slices' clips are virtual; the split-K mode runs no h3 conv
  q.y_amax = nullptr;
  const char* kname = "conv";
  HIPCHK(h, dcx::launch_conv(q, c.batch * S, w.phases, s, &kname));
  HIPCHK(h, dcx::launch_splitk_epilogue(p, h->split_buf, S, (long long)c.batch * p.y_bstride, c.batch, w.phases, s));
  ps.done((std::string("splitk:") + kname).c_str(), conv_flops(w, c), conv_bytes(w, c));
  return DCX_OK;
}

#ifdef DCX_DIAG_DUP
// Diagnostic builds: with DCX_DIAG_DUP=1 (no stores) or 2 (no epilogue) every conv launch is preceded
// by a timing copy on the same (real) inputs that writes nothing, profiled as "diag:<kernel>", so
// kernel tables compare each launch with and without its epilogue's stores on identical data.
int diag_dup_mode() {
  const char* e = std::getenv("DCX_DIAG_DUP");
  return e && (e[0] == '1' || e[0] == '2') ? e[0] - '0' : 0;
}
#endif

int run_conv(dcx_codec* h, const ConvW& w, const ConvCall& c, hipStream_t s, bool force_f32 = false) {
  ConvParams p;
  RUN(conv_params(h, w, c, force_f32, p));
  const int S = force_f32 ? 1 : split_factor(h, w, c, p);
  if (S > 1) return run_conv_split(h, w, c, p, S, s);
#ifdef DCX_DIAG_DUP
  if (const int dm = diag_dup_mode()) {
    ConvParams q = p;
    q.diag_skip = dm;
    ProfScope pd(h, s);
    const char* kn = "conv";
    HIPCHK(h, dcx::launch_conv(q, c.batch, w.phases, s, &kn));
    pd.done((std::string("diag:") + kn).c_str(), conv_flops(w, c), conv_bytes(w, c));
  }
#endif
  ProfScope ps(h, s);
  const char* kname = "conv";
  HIPCHK(h, dcx::launch_conv(p, c.batch, w.phases, s, &kname));
  ps.done(kname, conv_flops(w, c), conv_bytes(w, c));
  return DCX_OK;
}

// Split-K latency mode, grouped (round 4): the few-tile convs of one ResBlock dilation index (all
// three split-eligible) as ONE conv launch whose members get K-slice counts in proportion to their
// K (taps x chunks), within the CU count of workgroups, and ONE launch of their reduces, instead of
// two launches per conv (a C5 hop spent ~7 us per reduce launch, 107 of them).  Returns 1 when the
// group does not qualify (the caller splits the members one by one).
int run_conv_group_split(dcx_codec* h, const ConvW* const* w, const ConvCall* c, ConvParams* p, int n, double fl,
                         double by, hipStream_t s) {
  if (n < 2 || h->knobs.split_group_off) return 1;
  long long tiles[dcx::kMaxGroup], out[dcx::kMaxGroup], chunks[dcx::kMaxGroup];
  int S[dcx::kMaxGroup], smax[dcx::kMaxGroup];
  // a ParallelBlock's last convs (the mean folded into their epilogues) must all be split, so that
  // one reduce thread finishes every member of an element in ResBlock order
  const bool chain = p[0].mean_mode != dcx::MEAN_NONE;
  if (chain) {
    if (p[0].mean_mode != dcx::MEAN_FIRST || p[n - 1].mean_mode != dcx::MEAN_LAST) return 1;
    for (int i = 1; i < n - 1; ++i)
      if (p[i].mean_mode != dcx::MEAN_MID) return 1;
    for (int i = 1; i < n; ++i)
      if (p[i].macc != p[0].macc || c[i].Lq != c[0].Lq || w[i]->cout != w[0]->cout) return 1;
  }
  long long total = 0;
  for (int i = 0; i < n; ++i) {
    if (split_factor(h, *w[i], c[i], p[i]) < 2 || w[i]->taps < 3 || w[i]->out_mul != 1) return 1;
    tiles[i] = (long long)c[i].batch * ((c[i].Lq + 255) / 256) * (w[i]->cout / 128);
    out[i] = (long long)c[i].batch * p[i].y_bstride;
    const int unit = w[i]->taps % 2 ? 2 : 1;
    chunks[i] = (long long)w[i]->taps * (w[i]->cin / 16);
    // at most the handle's split_k slices per member (dcx_set_split_k), as split_factor allows
    smax[i] = (int)std::min<long long>(std::min(h->split_k, kSplitMax), (w[i]->cin / 16) / unit);
    S[i] = chain ? 2 : 1;
    if (S[i] > smax[i]) return 1;
    total += S[i] * tiles[i];
  }
  if (total > 256) return 1;
  // K slices: repeatedly give one more slice to the member whose slices are longest, while the
  // grid stays within one workgroup per CU
  for (;;) {
    int best = -1;
    for (int i = 0; i < n; ++i)
      if (S[i] < smax[i] && total + tiles[i] <= 256 &&
          (best < 0 || chunks[i] * S[best] > chunks[best] * S[i]))
        best = i;
    if (best < 0) break;
    ++S[best];
    total += tiles[best];
  }
  long long need = 0;
  for (int i = 0; i < n; ++i) need += S[i] > 1 ? S[i] * out[i] : 0;
  if (need > kSplitMax * kSplitMaxOut) return 1;
  ProfScope ps(h, s);
  ConvParams q[dcx::kMaxGroup], r[dcx::kMaxGroup];
  const float* part[dcx::kMaxGroup];
  int rs[dcx::kMaxGroup];
  long long rstride[dcx::kMaxGroup];
  int nr = 0;
  long long off = 0;
  for (int i = 0; i < n; ++i) {
    q[i] = p[i];
    q[i].ksplit = S[i];
    if (S[i] > 1) {  // partial sums into the split buffer, the epilogue in the reduce
      q[i].kunit = w[i]->taps % 2 ? 2 : 1;
      q[i].bias = q[i].gamma = q[i].res = nullptr;
      q[i].macc = nullptr;
      q[i].y = h->split_buf + off;
      q[i].y2 = nullptr;
      q[i].y6 = q[i].y6s = nullptr;
      q[i].epi = dcx::EPI_BIAS;
      q[i].mean_mode = dcx::MEAN_NONE;
      q[i].y_compact = 0;
      q[i].round_bf16 = 0;
      q[i].y_ash = nullptr;  // virtual clips (run_conv_split)
      q[i].y_amax = nullptr;
      r[nr] = p[i];
      part[nr] = h->split_buf + off;
      rs[nr] = S[i];
      rstride[nr] = out[i];
      ++nr;
      off += S[i] * out[i];
    }
  }
  const char* kname = "conv_group";
  const hipError_t e = dcx::launch_conv_split_group(q, n, c[0].batch, s, &kname);
  if (e == hipErrorNotSupported) return 1;
  HIPCHK(h, e);
  if (nr) HIPCHK(h, dcx::launch_splitk_epilogue_group(r, part, rs, rstride, nr, c[0].batch, chain, s));
  ps.done((std::string("splitk:") + kname).c_str(), fl, by);
  return DCX_OK;
}

// n independent convs (same batch) as one grouped launch when the kernel family allows it
// (dcx::launch_conv_group), otherwise one by one; the results are the same bits either way.
int run_conv_group(dcx_codec* h, const ConvW* const* w, const ConvCall* c, int n, hipStream_t s) {
  ConvParams p[dcx::kMaxGroup];
  double fl = 0, by = 0;
  bool same = true;
  for (int i = 0; i < n; ++i) {
    RUN(conv_params(h, *w[i], c[i], false, p[i]));
    fl += conv_flops(*w[i], c[i]);
    by += conv_bytes(*w[i], c[i]);
    same = same && c[i].batch == c[0].batch && w[i]->phases == 1;
  }
  if (same && n > 1 && h->split_k >= 2) {
    const int rc = run_conv_group_split(h, w, c, p, n, fl, by, s);
    if (rc != 1) return rc;
  }
  if (same && n > 1) {
#ifdef DCX_DIAG_DUP
    if (const int dm = diag_dup_mode()) {
      ConvParams q[dcx::kMaxGroup];
      for (int i = 0; i < n; ++i) {
        q[i] = p[i];
        q[i].diag_skip = dm;
      }
      ProfScope pd(h, s);
      const char* kn = "conv_group";
      const hipError_t e = dcx::launch_conv_group(q, n, c[0].batch, s, &kn);
      if (e == hipSuccess) pd.done((std::string("diag:") + kn).c_str(), fl, by);
    }
#endif
    ProfScope ps(h, s);
    const char* kname = "conv_group";
    const hipError_t e = dcx::launch_conv_group(p, n, c[0].batch, s, &kname);
    if (e == hipSuccess) {
      ps.done(kname, fl, by);
      return DCX_OK;
    }
    if (e != hipErrorNotSupported) HIPCHK(h, e);
  }
  for (int i = 0; i < n; ++i) RUN(run_conv(h, *w[i], c[i], s));
  return DCX_OK;
}

// Pointwise conv / Linear over all B*T rows at once.
ConvCall pointwise(CAct x, long long rows) {
  ConvCall c;
  c.x = x;
  c.x_bstride = 0;
  c.batch = 1;
  c.Lin = c.Lq = (int)rows;
  c.ldx = 0;
  return c;
}
ConvCall framed(CAct x, int B, int L, int C) {
  ConvCall c;
  c.x = x;
  c.x_bstride = (long long)L * C;
  c.batch = B;
  c.Lin = c.Lq = L;
  c.ldx = C;
  return c;
}


#define LAUNCH(h, s, name, flops, bytes, expr) \
  do {                                         \
    ProfScope ps_(h, s);                       \
    HIPCHK(h, expr);                           \
    ps_.done(name, flops, bytes);              \
  } while (0)

// fp32 -> planes (or, with compact, bf16) for a tensor handed in by the caller (x6 / bf16 modes).
// h2: the h2 layout instead (an h3 consumer; a planes tensor handed in with its fp32 copy is re-split),
// range-scaled (dcx_kernels.h h2_shift) by the exact max of each clip (`clips` clips of rows / clips
// rows: launch_h2_ranged, for the tap convs) or, with clips == 0, of each row (launch_h2_rows, for the
// one-tap convs).  The scale follows from the values alone, so a tensor the fused pipeline would have
// produced in h2 itself (a LayerNorm's row-scaled output) gets the same bits here.
int ensure_planes(dcx_codec* h, CAct& a, long long rows, int C, Bump& ws, hipStream_t s, bool compact = false,
                  bool h2 = false, int clips = 0) {
  if (h2 && a.p && !a.h2 && a.f) a.p = nullptr;
  if (!x6_mode(h) || a.p) return DCX_OK;
  const bool rh2 = h2 && !compact;
  unsigned short* p = ws.u16((size_t)rows * C * 3);
  float* am = rh2 && clips ? ws.f((size_t)clips) : nullptr;
  int* ash = rh2 ? ws.i((size_t)(clips ? clips : rows)) : nullptr;
  if (ws.dry) return DCX_OK;
  if (!ws.ok()) return fail(h, DCX_ERR_WORKSPACE, "workspace too small");
  if (rh2 && clips) {
    if (clips < 1 || rows % clips) return fail(h, DCX_ERR_STATE, "internal: ranged split of a ragged batch");
    LAUNCH(h, s, "h2_ranged", 0, 12.0 * rows * C,
           dcx::launch_h2_ranged(a.f, nullptr, p, clips, rows / clips, C, 0, 0.f, am, ash, h->rflag, s));
    a.r = Rng{};
    a.r.ash = ash;
    a.r.amax = am;
  } else if (rh2) {
    LAUNCH(h, s, "h2_rows", 0, 8.0 * rows * C, dcx::launch_h2_rows(a.f, p, rows, C, ash, s));
    a.r = Rng{};
    a.r.ash_row = ash;
  } else {
    LAUNCH(h, s, "split_planes", 0, (compact ? 6.0 : 10.0) * rows * C,
           dcx::launch_split_planes(a.f, p, rows, C, compact ? 1 : 0, s));
  }
  a.p = p;
  a.c1 = compact;
  a.h2 = rh2;
  return DCX_OK;
}

// ConvNeXtBlock in place on x [B][T][C] (fp32 residual stream); out6: optional planes (compact
// with out6c) of the block output for a following conv.  ln: [M][C], hid: [M][4C] conv-input
// scratch, written compact where their consumer takes it (bf16 mode).
// ConvNeXtBlock in place on x [B][T][C] (fp32 residual stream); out6: optional planes (compact
// with out6c = 1) of the block output for a following conv.  ln: [M][C], hid: [M][4C] conv-input
// scratch, written compact where their consumer takes it (bf16 mode), or in h2 with per-row ranges
// (ln.row_ash / row_amax, hid.row_ash: the LayerNorm's exact row maxima, the hidden's rows bounded
// by g1 max|LN row| + max|b1|; round 6).
int run_block(dcx_codec* h, const BlockW& bw, float* x, unsigned short* out6, int B, int T, Act ln, Act hid,
              hipStream_t s, int out6c = 0) {
  const long long M = (long long)B * T;
  const int C = bw.C;
  if (out6 && out6c == 3) return fail(h, DCX_ERR_STATE, "internal: a block output in h2 goes through launch_h2_rows");
  ln.c1 = ln.p && takes_compact(h, bw.pw1, M);
  hid.c1 = hid.p && takes_compact(h, bw.pw2, M);
  ln.h2 = ln.p && ln.row_ash && ln.row_amax && takes_h3(h, bw.pw1);
  hid.h2 = hid.p && hid.row_ash && takes_h3(h, bw.pw2);
  ln.r = Rng{};
  hid.r = Rng{};
  ln.r.ash_row = ln.row_ash;
  hid.r.ash_row = hid.row_ash;
  LAUNCH(h, s, "dwconv_ln", 14.0 * M * C, 8.0 * M * C,
         dcx::launch_dwconv_ln(x, ln.f, ln.p, ln.c1 ? 1 : ln.h2 ? 3 : 0, bw.dww, bw.dwb, bw.ln.w, bw.ln.b, B, T, C,
                               h->gemm_mode == DCX_GEMM_BF16 ? 1 : 0, &h->knobs, s, ln.row_ash, ln.row_amax));
  ConvCall c1 = pointwise(ln, M);
  c1.out_to(hid);
  c1.epi = dcx::EPI_GELU;
  if (hid.h2) {  // |GELU(v)| <= |v| <= g1 max|LN row| + max|b1|
    c1.yb = prog_conv_rows(bw.pw1, ln.row_amax);
    c1.y_ash = hid.row_ash;
  }
  RUN(run_conv(h, bw.pw1, c1, s));
  ConvCall c2 = pointwise(hid, M);
  c2.y = x;
  c2.y6 = out6;
  c2.y6c = out6 ? out6c : 0;  // 0 planes, 1 compact
  c2.res = x;
  c2.gamma = bw.gamma;
  c2.epi = dcx::EPI_GAMMA_RES;
  RUN(run_conv(h, bw.pw2, c2, s));
  return DCX_OK;
}

// channels-first LayerNorm; bf16_in: its input is a bf16 tensor under the reference's autocast (the
// stem's, in bf16 mode), so its mean and differences are bf16 (ln_rows form 2).  An h2 output (y.h2)
// is scaled per row by its exact max (y.row_ash receives the shifts, y.row_amax the maxima if set).
int run_ln(dcx_codec* h, const LnW& l, const float* x, Act y, long long rows, hipStream_t s, bool bf16_in = false) {
  const int form = bf16_in && h->gemm_mode == DCX_GEMM_BF16 ? 2 : 1;
  if (y.p && y.h2 && !y.row_ash) return fail(h, DCX_ERR_STATE, "internal: h2 LayerNorm output without row ranges");
  LAUNCH(h, s, "ln_rows", 8.0 * rows * l.C, 8.0 * rows * l.C,
         dcx::launch_ln_rows(x, y.f, y.p, y.p && y.c1 ? 1 : y.p && y.h2 ? 3 : 0, l.w, l.b, rows, l.C, 1e-6f, form, s,
                             y.row_ash, y.row_amax));
  return DCX_OK;
}

// Per-row range buffers for the block scratch of M rows (x6 mode only: the h3 one-tap convs).
void row_ranges(dcx_codec* h, Bump& ws, long long M, Act& ln, Act& hid) {
  if (!x6_mode(h)) return;
  ln.row_ash = ws.i((size_t)M);
  ln.row_amax = ws.f((size_t)M);
  hid.row_ash = ws.i((size_t)M);
}

// ---------------- stage bodies (dry=true only sizes the workspace) ----------------
int stage_mel(dcx_codec* h, const float* audio, int B, int64_t n, Act mel, Bump& ws, hipStream_t s,
              float* loglin = nullptr) {
  const dcx_config& c = h->cfg;
  const int T = (int)frames_of(c, n);
  const int rows = T + c.n_fft / c.hop - 1;
  Act fr = conv_input(h, ws, (size_t)B * rows * c.hop);
  float* spec = ws.f((size_t)B * T * h->dft.cout);
  Act mag = conv_input(h, ws, (size_t)B * T * h->melfb.cin);
  if (ws.dry) return DCX_OK;
  if (!ws.ok()) return fail(h, DCX_ERR_WORKSPACE, "workspace too small for mel");
  LAUNCH(h, s, "frame_pad", 0, 8.0 * B * rows * c.hop,
         dcx::launch_frame_pad(audio, fr.f, fr.p, B, n, rows, c.hop, (c.win - c.hop) / 2, s));
  ConvCall cc = framed(fr, B, rows, c.hop);
  cc.exact = true;
  cc.Lq = T;
  cc.y = spec;
  RUN(run_conv(h, h->dft, cc, s));
  const int nbins = c.n_fft / 2 + 1;
  LAUNCH(h, s, "spec_mag", 4.0 * B * T * nbins, 4.0 * B * T * (h->dft.cout + h->melfb.cin),
         dcx::launch_spec_mag(spec, mag.f, mag.p, loglin, (long long)B * T, nbins, h->melfb.cin, s));
  ConvCall cm = pointwise(mag, (long long)B * T);
  cm.exact = true;
  cm.out_to(mel);
  cm.epi = dcx::EPI_LOGCLAMP;
  RUN(run_conv(h, h->melfb, cm, s));
  return DCX_OK;
}

// Whether a call may fork its half-batches onto the side stream: a handle with one, not inside a
// half already, and a caller's stream that is not being captured into a hipGraph (a captured call
// keeps to the caller's stream, with the same bits)
bool may_fork(dcx_codec* h, hipStream_t s) {
  if (!h->side || h->no_fork) return false;
  hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
  return hipStreamIsCapturing(s, &st) == hipSuccess && st == hipStreamCaptureStatusNone;
}

// Rows [r0, ...) (clips b0 on) of a [B][T][C] activation in its layout (planes 3, h2 2, compact 1
// ushorts per element), with its per-row and per-clip range pointers.
template <class A>
A act_rows(A a, int b0, long long r0, long long C) {
  if (a.f) a.f += r0 * C;
  if (a.p) a.p += r0 * C * (a.c1 ? 1 : a.h2 ? 2 : 3);
  if (a.r.ash) a.r.ash += b0;
  if (a.r.amax) a.r.amax += b0;
  if (a.r.ash_row) a.r.ash_row += r0;
  return a;
}
Act act_rows_out(Act a, int b0, long long r0, long long C) {
  a = act_rows(a, b0, r0, C);
  if (a.row_ash) a.row_ash += r0;
  if (a.row_amax) a.row_amax += r0;
  return a;
}
// A conv-input scratch region (conv_input: planes-sized) of n elements per row, from row r0 on.
Act scratch_rows(Act a, long long r0, long long n) {
  if (a.f) a.f += r0 * n;
  if (a.p) a.p += r0 * n * 3;
  if (a.row_ash) a.row_ash += r0;
  if (a.row_amax) a.row_amax += r0;
  return a;
}

// The encoder (encoders.py:68-76) on clips of one batch: stem conv + LN, 4 stages of (LN +
// downsample 1x1 conv) and ConvNeXt blocks, the final LayerNorm into feat.
int encode_clips(dcx_codec* h, const CAct& mel, int B, int T, Act feat, float* xa, float* xb, Act ln, Act hid,
                 hipStream_t s) {
  const dcx_config& c = h->cfg;
  const long long M = (long long)B * T;
  ConvCall cc = framed(mel, B, T, c.n_mels);
  cc.y = xa;
  RUN(run_conv(h, h->stem, cc, s));
  RUN(run_ln(h, h->stem_ln, xa, Act{xb, nullptr}, M, s, /*bf16_in=*/true));
  for (int i = 0; i < 4; ++i) {
    if (i > 0) {
      ln.c1 = ln.p && takes_compact(h, h->ds_conv[i], M);
      ln.h2 = ln.p && ln.row_ash && takes_h3(h, h->ds_conv[i]);  // the downsample 1x1 conv on conv_gemm_x3dw
      ln.r = Rng{};
      ln.r.ash_row = ln.h2 ? ln.row_ash : nullptr;  // row-scaled by run_ln
      RUN(run_ln(h, h->ds_ln[i], xb, ln, M, s));
      ConvCall cd = pointwise(ln, M);
      cd.y = xb;
      RUN(run_conv(h, h->ds_conv[i], cd, s));
    }
    for (auto& bw : h->blocks[i]) RUN(run_block(h, bw, xb, nullptr, B, T, ln, hid, s));
  }
  RUN(run_ln(h, h->enc_norm, xb, feat, M, s));  // an h2 feat: row-scaled into feat.row_ash
  return DCX_OK;
}

// Two half-batches on two streams (round 6, Knobs::enc_streams): the encoder's launches are short
// (the 1x1 convs of a C2 batch are 0.5-7 rounds of tiles over the CUs, e.g. pwconv2 at C = 768:
// 354 tiles = 1.38 rounds), so one half's partly filled last round runs beside the other half's
// launches.  Every kernel computes a clip's rows alone (tiles never span clips; per-row range
// scales), so the halves give the bits of the whole batch.
int stage_encode(dcx_codec* h, CAct mel, int B, int T, Act feat, Bump& ws, hipStream_t s) {
  const dcx_config& c = h->cfg;
  const long long M = (long long)B * T;
  const int cmax = c.enc_dims[3];
  RUN(ensure_planes(h, mel, M, c.n_mels, ws, s));
  float* xa = ws.f((size_t)M * cmax);
  float* xb = ws.f((size_t)M * cmax);
  Act ln = conv_input(h, ws, (size_t)M * cmax);
  Act hid = conv_input(h, ws, (size_t)M * 4 * cmax);
  row_ranges(h, ws, M, ln, hid);
  if (ws.dry) return DCX_OK;
  if (!ws.ok()) return fail(h, DCX_ERR_WORKSPACE, "workspace too small for encode");
  if (B < 2 || !h->knobs.enc_streams || !may_fork(h, s)) return encode_clips(h, mel, B, T, feat, xa, xb, ln, hid, s);
  const int B0 = (B + 1) / 2;
  const long long r1 = (long long)B0 * T;
  HIPCHK(h, hipEventRecord(h->fork_ev, s));
  HIPCHK(h, hipStreamWaitEvent(h->side, h->fork_ev, 0));
  const int rc0 = encode_clips(h, mel, B0, T, feat, xa, xb, ln, hid, s);
  const int rc1 = rc0 != DCX_OK ? rc0
                                : encode_clips(h, act_rows(mel, B0, r1, c.n_mels), B - B0, T,
                                               act_rows_out(feat, B0, r1, cmax), xa + r1 * cmax, xb + r1 * cmax,
                                               scratch_rows(ln, r1, cmax), scratch_rows(hid, r1, 4LL * cmax), h->side);
  // joined whatever happened, so the caller's stream never runs ahead of the side stream's work
  const hipError_t e0 = hipEventRecord(h->join_ev, h->side);
  const hipError_t e1 = hipStreamWaitEvent(s, h->join_ev, 0);
  RUN(rc1);
  HIPCHK(h, e0);
  HIPCHK(h, e1);
  return DCX_OK;
}

// x_pjt_in layout the nearest-code search reads (ConvParams::x_compact): 1 compact bf16 for
// vq_prefilter_b1 (x6 and bf16 modes), else 0 planes (vq_prefilter_x3 / _dm; fp32 mode ignores it).
// DCX_VQ_OLD builds (A/B): 1 in bf16 mode (vq_prefilter_bq), 2 "hm" in x6 mode (vq_prefilter_dm).
int vq_xlayout(const dcx_codec* h, long long M) {
  if (!x6_mode(h) || !h->compact) return 0;
#ifdef DCX_VQ_OLD
  if (!h->codebook_bk) return 0;
  if (h->gemm_mode == DCX_GEMM_BF16) return 1;
  return dcx::vq_hm_takes(h->cfg.codebook_size, h->cfg.codebook_dim, M) ? 2 : 0;
#else
  (void)M;
  return h->codebook_b1 ? 1 : 0;
#endif
}

// The nearest-code search of DownsampleGRVQ (vector_quantize_pytorch.py:41-45, 496-506; first index on
// ties) on x_pjt_in P (fp32 [M][CD]) and, in x6 / bf16 mode, P6 in the prefilter's layout xl (0 planes,
// 1 compact bf16, 2 hm): |x|^2, the certified prefilter and the fp64 rescore (x6 / bf16), or the exact
// fp32 distance GEMM and its reduce (fp32 mode).  pv / pi / pv2: [M][ntiles] scratch, x2: [M].
// Workspace of one search of M rows: the prefilter's [M][ntiles] partials and, in x6 / bf16 mode, the
// rescore's candidate list (128 pairs per row on average: the C2 workload lists 62 in x6 mode; a row that does not fit is rescored in place).
struct VqScratch {
  float *x2 = nullptr, *xr2 = nullptr, *pv = nullptr, *pv2 = nullptr;
  int* pi = nullptr;
  double *x2d = nullptr, *cdist = nullptr;
  int* ccode = nullptr;
  int2 *pairs = nullptr, *row_list = nullptr;
  unsigned long long* npairs = nullptr;
  long long cap = 0;
};
VqScratch vq_scratch(const dcx_codec* h, Bump& ws, long long M, int ntiles, bool x6) {
  VqScratch v;
  v.x2 = ws.f((size_t)M);
  v.pv = ws.f((size_t)M * ntiles);
  v.pi = ws.i((size_t)M * ntiles);
  if (x6) {
    v.xr2 = ws.f((size_t)M);
    v.pv2 = ws.f((size_t)M * ntiles);
    v.x2d = (double*)ws.raw((size_t)M * sizeof(double));
    // list offsets are stored as int (row_list): at most INT_MAX pairs; rows beyond are rescored in place
    v.cap = h->vq_pairs_per_row > 0
                ? std::min<long long>(std::max<long long>((long long)h->vq_pairs_per_row * M, 1024), INT_MAX) / 8 * 8
                : 0;
    v.pairs = (int2*)ws.raw((size_t)v.cap * sizeof(int2));
    v.cdist = (double*)ws.raw((size_t)(v.cap / 8) * sizeof(double));
    v.ccode = ws.i((size_t)(v.cap / 8));
    v.row_list = (int2*)ws.raw((size_t)M * sizeof(int2));
    v.npairs = (unsigned long long*)ws.raw(sizeof(unsigned long long));
  }
  return v;
}

int run_vq_search(dcx_codec* h, const float* P, const unsigned short* P6, int xl, long long M, const VqScratch& v,
                  int ntiles, int32_t* codes, hipStream_t s) {
  const dcx_config& c = h->cfg;
  const int CD = c.codebook_dim, NC = c.codebook_size;
  const bool x6 = x6_mode(h);
  const bool p6c = xl == 1, p6hm = xl == 2;
  const bool b1 = p6c && dcx::vq_b1_takes(NC, CD);
  float* const x2 = v.x2;
  LAUNCH(h, s, "row_sqnorm", 2.0 * M * CD, 4.0 * M * CD,
         dcx::launch_row_sqnorm(P, M, CD, x2, x6 ? v.x2d : nullptr, b1 ? v.xr2 : nullptr, x6 ? v.npairs : nullptr, s));
  {
    ConvParams p{};
    p.x = P; p.x6 = P6; p.w = h->codebook; p.w6 = x6 ? h->codebook6 : nullptr;
    p.Cin = CD; p.Cout = NC; p.ldx = CD; p.taps = 1; p.in_step = 1; p.out_mul = 1;
    p.x2 = x2; p.e2 = h->e2; p.part_val = v.pv; p.part_idx = v.pi; p.part_val2 = v.pv2;
    p.x_compact = p6c ? 1 : p6hm ? 2 : 0;
    p.wc = b1 ? h->codebook_b1 : p6c || p6hm ? h->codebook_bk : nullptr;
    ProfScope ps(h, s);
    const char* kname = "vq";
    if (x6) {
      // bf16 mode rounds x_pjt_in to bf16 in the project_in epilogue (round_bf16)
      HIPCHK(h, dcx::launch_vq_prefilter(p, (int)M, h->gemm_mode == DCX_GEMM_BF16, s, &kname));
      ps.done(kname, 2.0 * M * NC * CD, 4.0 * ((double)M * CD + (double)NC * CD));
    } else {
      HIPCHK(h, dcx::launch_vq_argmin(p, (int)M, s, &kname));
      ps.done(kname, 2.0 * M * NC * CD, 4.0 * ((double)M * CD + (double)NC * CD));
    }
  }
  if (x6) {
    dcx::VqRescoreArgs a{};
    a.part_val = v.pv; a.part_val2 = v.pv2; a.part_idx = v.pi;
    a.rows = M; a.ntiles = ntiles; a.tile_codes = NC / ntiles; a.dim = CD;
    a.x = P; a.x2 = x2; a.xr2 = b1 ? v.xr2 : nullptr; a.x2d = v.x2d;
    a.codebook = h->codebook; a.e2d = h->e2d;
    a.cx = dcx::vq_prefilter_cx(xl, NC, CD, h->emax, h->dmax); a.emax = h->emax; a.e2max = h->e2max;
    a.codes = codes; a.stats = h->vq_stats_on ? h->vq_stats : nullptr;
    a.pairs = v.pairs; a.cdist = v.cdist; a.ccode = v.ccode; a.cap = v.cap; a.row_list = v.row_list; a.npairs = v.npairs;
    LAUNCH(h, s, "vq_certify", 0, 12.0 * M * ntiles + 4.0 * M, dcx::launch_vq_certify(a, s));
    LAUNCH(h, s, "vq_pair_eval", 0, 0, dcx::launch_vq_pair_eval(a, s));
    LAUNCH(h, s, "vq_pair_reduce", 0, 0, dcx::launch_vq_pair_reduce(a, s));
  } else {
    LAUNCH(h, s, "vq_reduce", 0, 8.0 * M * ntiles, dcx::launch_vq_reduce(v.pv, v.pi, (int)M, ntiles, codes, s));
  }
  return DCX_OK;
}

// decode table in planes for this mode's gathers: project_out in fp32 (x6) or under autocast (bf16)
const unsigned short* decode_table6(const dcx_codec* h) {
  return h->gemm_mode == DCX_GEMM_BF16 && h->ptable6b ? h->ptable6b : h->ptable6;
}

int stage_vq_encode(dcx_codec* h, CAct feat, int B, int T, int32_t* codes, float* pin, float* fup, float* quant,
                    Bump& ws, hipStream_t s) {
  const dcx_config& c = h->cfg;
  const long long M = (long long)B * T;
  const int D = c.vq_dim, CD = c.codebook_dim, NC = c.codebook_size;
  const bool x6 = x6_mode(h);
  const int xl = vq_xlayout(h, M);
  const int ntiles = x6 ? dcx::vq_prefilter_ntiles(NC, CD, M, xl) : dcx::vq_argmin_ntiles(NC);
  // the down conv's input as the fused pipeline writes it: compact bf16 (bf16 mode) or h2 (h3), the
  // latter scaled per row by the row's exact max as the encoder's final LayerNorm scales it, so the
  // staged and the fused call compute the same bits
  {
    const bool cmp = takes_compact(h, h->vq_down, M);
    RUN(ensure_planes(h, feat, M, D, ws, s, cmp, !cmp && takes_h3(h, h->vq_down), 0));
  }
  if (feat.c1 && !takes_compact(h, h->vq_down, M)) return fail(h, DCX_ERR_STATE, "internal: compact features");
  float* X = ws.f((size_t)M * D);
  unsigned short* X6 = x6 ? ws.u16((size_t)M * D * 3) : nullptr;
  Act ln = conv_input(h, ws, (size_t)M * D);
  Act hid = conv_input(h, ws, (size_t)M * 4 * D);
  row_ranges(h, ws, M, ln, hid);
  int* x6_ash = x6 ? ws.i((size_t)M) : nullptr;  // project_in's input rows' shifts (h3)
  float* P = pin ? pin : ws.f((size_t)M * CD);
  unsigned short* P6 = x6 ? ws.u16((size_t)M * CD * 3) : nullptr;
  const VqScratch vs = vq_scratch(h, ws, M, ntiles, x6);
  Act zd = conv_input(h, ws, (size_t)M * D);
  if (ws.dry) return DCX_OK;
  if (!ws.ok()) return fail(h, DCX_ERR_WORKSPACE, "workspace too small for vq_encode");
  ConvCall cd = pointwise(feat, M);
  cd.y = X;
  RUN(run_conv(h, h->vq_down, cd, s));
  const bool x6c = X6 && takes_compact(h, h->vq_pin, M);
  const bool h2p = X6 && !x6c && takes_h3(h, h->vq_pin);  // project_in on conv_gemm_x3dw
  // the block's output for project_in: compact / planes from its epilogue, or (h3) split per row by
  // the row's exact max afterwards (launch_h2_rows)
  RUN(run_block(h, h->vq_down_blk, X, h2p ? nullptr : X6, B, T, ln, hid, s, x6c ? 1 : 0));
  if (h2p) LAUNCH(h, s, "h2_rows", 0, 8.0 * M * D, dcx::launch_h2_rows(X, X6, M, D, x6_ash, s));
  CAct pin_in(X, X6, x6c);
  pin_in.h2 = h2p;
  if (h2p) pin_in.r.ash_row = x6_ash;
  ConvCall cp = pointwise(pin_in, M);
  cp.y = P;
  cp.y6 = P6;
  cp.y6c = xl;
  RUN(run_conv(h, h->vq_pin, cp, s));
  RUN(run_vq_search(h, P, P6, xl, M, vs, ntiles, codes, s));
  if (fup) LAUNCH(h, s, "gather_rows", 0, 8.0 * M * CD, dcx::launch_gather_rows(h->codebook, NC, codes, M, CD, fup, nullptr, -1, s));
  if (quant) {
    if (x6)
      LAUNCH(h, s, "gather_rows", 0, 12.0 * M * D,
             dcx::launch_gather_rows((const float*)decode_table6(h), NC, codes, M, D * 3 / 2, (float*)zd.p, nullptr, NC, s));
    else
      LAUNCH(h, s, "gather_rows", 0, 8.0 * M * D, dcx::launch_gather_rows(h->ptable, NC, codes, M, D, zd.f, nullptr, NC, s));
    ConvCall cu = pointwise(zd, M);
    cu.y = quant;
    RUN(run_conv(h, h->vq_up, cu, s));
    RUN(run_block(h, h->vq_up_blk, quant, nullptr, B, T, ln, hid, s));
  }
  return DCX_OK;
}

// z.f is required (fp32 residual stream of the up-path block); z.p optionally receives planes.
int stage_vq_decode(dcx_codec* h, const int32_t* codes, int B, int T, Act z, int32_t* n_invalid, Bump& ws,
                    hipStream_t s) {
  const dcx_config& c = h->cfg;
  const long long M = (long long)B * T;
  const int D = c.vq_dim;
  Act zd = conv_input(h, ws, (size_t)M * D);
  Act ln = conv_input(h, ws, (size_t)M * D);
  Act hid = conv_input(h, ws, (size_t)M * 4 * D);
  row_ranges(h, ws, M, ln, hid);
  if (ws.dry) return DCX_OK;
  if (!ws.ok()) return fail(h, DCX_ERR_WORKSPACE, "workspace too small for vq_decode");
  if (z.p && z.h2) return fail(h, DCX_ERR_STATE, "internal: z in h2 is split by the generator (ranged per clip)");
  if (x6_mode(h))
    LAUNCH(h, s, "gather_rows", 0, 12.0 * M * D,
           dcx::launch_gather_rows((const float*)decode_table6(h), c.codebook_size, codes, M, D * 3 / 2, (float*)zd.p,
                                   n_invalid, c.codebook_size, s));
  else
    LAUNCH(h, s, "gather_rows", 0, 8.0 * M * D,
           dcx::launch_gather_rows(h->ptable, c.codebook_size, codes, M, D, zd.f, n_invalid, c.codebook_size, s));
  ConvCall cu = pointwise(zd, M);
  cu.y = z.f;
  RUN(run_conv(h, h->vq_up, cu, s));
  RUN(run_block(h, h->vq_up_blk, z.f, z.p, B, T, ln, hid, s));
  return DCX_OK;
}

// The fused pair kernel serves a stage when its ResBlock convs are C = 32 / 64 in x6 arithmetic with
// odd kernels, c2 reach <= 8 and c1 reach <= 32 rows, and biases (launch_res_pair checks again).
bool res_pair_ok(const dcx_codec* h, int stage) {
  if (!h->res_pair || h->gemm_mode != DCX_GEMM_X6) return false;
  const dcx_config& c = h->cfg;
  for (int rb = 0; rb < c.n_res; ++rb)
    for (int ci = 0; ci < 3; ++ci)
      for (int j = 0; j < 2; ++j) {
        const ConvW& w = h->res[stage][rb][ci][j];
        const int hk = (w.taps - 1) / 2;
        if ((w.cout != 32 && w.cout != 64) || w.cin != w.cout || !w.w6 || !w.b || w.taps % 2 == 0 || hk > 8 ||
            w.phases != 1 || w.in_step < 1 || hk * w.in_step > 32 || w.in_base[0] != -hk * w.in_step ||
            (j == 1 && w.in_step != 1))
          return false;
      }
  return true;
}

// Whether generator stage i runs its ResBlock convs in h3 arithmetic (Knobs::h3, x6 mode, not in
// the split-K latency mode, every conv with h3 weights): their inputs are then written in the h2
// layout by their producers (ConvT, c1, c2 epilogues).
// rows: the stage's rows per clip (its ResBlock convs' input length)
bool h3_stage(const dcx_codec* h, int i, long long rows) {
  if (!h->knobs.h3 || h->gemm_mode != DCX_GEMM_X6 || h->split_k >= 2) return false;
  if (!h3_rows_ok(rows, h->res[i][0][0][0].cin)) return false;
  for (int rb = 0; rb < h->cfg.n_res; ++rb)
    for (int j = 0; j < 3; ++j)
      if (!h->res[i][rb][j][0].w3 || !h->res[i][rb][j][1].w3) return false;
  return true;
}

// Buffers of one generator stage's ParallelBlock (run_parallel_block).
struct PBlockBufs {
  float* X = nullptr;                // ConvT output: the ResBlocks' input (fp32)
  Act XS;                            // silu(X) in the c1 convs' input form (unused when silu is applied on load)
  float* R[dcx::kMaxGroup] = {};     // ResBlock states (fp32)
  Act RS[dcx::kMaxGroup];            // silu(R), c1 input form
  Act Tb[dcx::kMaxGroup];            // silu(c1 output) buffers as allocated
  Act Tb_in[dcx::kMaxGroup];         // the same in the c2 convs' input form
  float* Mx = nullptr;               // mean accumulator; silu(mean) in fp32 when `last`
  Act next;                          // silu(mean) in the next ConvT's input form (not `last`)
  bool last = false;
  // h3 ranges (round 6): the measured per-clip max |X| (XS.r carries its h2 shift), the slots that
  // receive the mean's max |.| and h2 shift (not `last`), and the call's slots for everything else
  const float* amax_X = nullptr;
  float* next_amax = nullptr;
  int* next_ash = nullptr;
  RangeArena* ra = nullptr;
};

// ParralelBlock.forward (convnext_utils.py:137-138) of generator stage i: three ResBlock1
// (convnext_utils.py:106-113) on X, their mean, and the SiLU that follows it in the generator
// (generators.py:125 / :141), written to b.Mx as fp32 (b.last) or to b.next.  The C = 32 / 64
// stages run as fused pairs (conv_res_pair), the others as grouped per-conv launches.  Every h2
// tensor is range-scaled from a bound over the maxima its producers measured (dcx_kernels.h).
int run_parallel_block(dcx_codec* h, int i, int B, int Lo, const PBlockBufs& b, hipStream_t s) {
  const dcx_config& c = h->cfg;
  constexpr int NR = dcx::kMaxGroup;
  const ConvW& rconv = h->res[i][0][0][0];  // every ResBlock conv of the stage has Cin = Cout = Co
  const int Co = rconv.cout;
  const bool silu_on_load = x6_mode(h) && f32_input_ok(rconv);
  RangeArena& ra = *b.ra;
  if (silu_on_load && res_pair_ok(h, i)) {
    // fused pairs: X -> R[rb] -> Tb[rb] (as fp32) -> silu(ParallelBlock mean)
    float* Ra[NR];
    float* Rb[NR];
    for (int rb = 0; rb < c.n_res; ++rb) {
      Ra[rb] = b.R[rb];
      Rb[rb] = b.Tb[rb].f ? b.Tb[rb].f : reinterpret_cast<float*>(b.Tb[rb].p);
    }
    float* out = b.last ? b.Mx : b.next.f;
    bool h3 = h->knobs.h3_pairs && h->split_k < 2;  // conv_res_pair_h3 (every conv with h3 weights)
    for (int rb = 0; rb < c.n_res; ++rb)
      for (int ci = 0; ci < 3; ++ci) h3 = h3 && h->res[i][rb][ci][0].w3 && h->res[i][rb][ci][1].w3;
    const float* st_amax[NR];  // measured max |state| per clip of each ResBlock's pair input
    for (int rb = 0; rb < c.n_res; ++rb) st_amax[rb] = b.amax_X;
    for (int ci = 0; ci < 3; ++ci) {
      dcx::ResPairParams rp{};
      rp.h3 = h3 ? 1 : 0;
      double fl = 0, by = 0;
      for (int rb = 0; rb < c.n_res; ++rb) {
        const ConvW& w1 = h->res[i][rb][ci][0];
        const ConvW& w2 = h->res[i][rb][ci][1];
        rp.src[rb] = ci == 0 ? b.X : (ci == 1 ? Ra[rb] : Rb[rb]);
        rp.dst[rb] = ci == 0 ? Ra[rb] : (ci == 1 ? Rb[rb] : nullptr);
        rp.w1[rb] = h3 ? w1.w3 : w1.w6;
        rp.w2[rb] = h3 ? w2.w3 : w2.w6;
        rp.w3_shift1[rb] = w1.w3_shift;
        rp.w3_shift2[rb] = w2.w3_shift;
        rp.b1[rb] = w1.b;
        rp.b2[rb] = w2.b;
        rp.taps[rb] = w1.taps;
        rp.dil[rb] = w1.in_step;
        rp.src_amax[rb] = st_amax[rb];
        rp.dst_amax[rb] = ci < 2 ? ra.amax() : nullptr;
        rp.g1[rb] = w1.g_abs;
        rp.bm1[rb] = w1.b_abs;
        ConvCall cc = framed(Act{b.X, nullptr}, B, Lo, Co);
        fl += conv_flops(w1, cc) + conv_flops(w2, cc);
        by += 8.0 * B * Lo * Co;
      }
      rp.nmem = c.n_res;
      rp.mean_out = ci == 2 ? out : nullptr;
      rp.bstride = (long long)Lo * Co;
      rp.L = Lo;
      rp.batch = B;
      rp.C = Co;
      rp.rflag = h->rflag;
      rp.kn = &h->knobs;
      if (h3)
        for (int rb = 0; rb < c.n_res; ++rb)
          if (!rp.src_amax[rb] || (ci < 2 && !rp.dst_amax[rb]))
            return fail(h, DCX_ERR_STATE, "internal: h3 range slots exhausted");
      ProfScope ps(h, s);
      const char* kname = "conv_res_pair";
      HIPCHK(h, dcx::launch_res_pair(rp, s, &kname));
      ps.done(kname, fl, by);
      for (int rb = 0; rb < c.n_res; ++rb) st_amax[rb] = rp.dst_amax[rb];
    }
    return DCX_OK;
  }
  // ranges of each ResBlock's state (its max |.|) and of the c1 inputs in h2
  Rng st[NR], in1[NR];
  for (int rb = 0; rb < c.n_res; ++rb) {
    st[rb].amax = b.amax_X;
    in1[rb] = b.XS.r;
    in1[rb].amax = b.amax_X;
  }
  for (int ci = 0; ci < 3; ++ci) {
    const ConvW* w1[NR];
    ConvCall c1[NR];
    Rng tr[NR];  // silu(c1 output): shift and the measured max |c1 output|
    for (int rb = 0; rb < c.n_res; ++rb) {  // c1 of every ResBlock: one grouped launch
      Act src = silu_on_load ? Act{ci == 0 ? b.X : b.R[rb], nullptr} : (ci == 0 ? b.XS : b.RS[rb]);
      src.r = in1[rb];
      c1[rb] = framed(src, B, Lo, Co);
      c1[rb].silu_in = silu_on_load;
      c1[rb].silu_to(b.Tb_in[rb]);
      w1[rb] = &h->res[i][rb][ci][0];
      c1[rb].yb = prog_conv(*w1[rb], in1[rb]);
      c1[rb].y_amax = ra.amax();
      c1[rb].y_ash = b.Tb_in[rb].h2 ? ra.ash() : nullptr;
      tr[rb].ash = c1[rb].y_ash;
      tr[rb].amax = c1[rb].y_amax;
    }
    RUN(run_conv_group(h, w1, c1, c.n_res, s));
    if (ci < 2) {  // c2 of every ResBlock: grouped; residual X (first pair) or the block's state
      const ConvW* w2[NR];
      ConvCall c2[NR];
      for (int rb = 0; rb < c.n_res; ++rb) {
        Act tin = b.Tb_in[rb];
        tin.r = tr[rb];
        c2[rb] = framed(tin, B, Lo, Co);
        c2[rb].epi = dcx::EPI_RES;
        c2[rb].res = ci == 0 ? b.X : b.R[rb];
        c2[rb].y = b.R[rb];
        if (!silu_on_load) c2[rb].silu_to(b.RS[rb]);
        w2[rb] = &h->res[i][rb][ci][1];
        // |state + c2 + b2| <= max|state| + g2 max|c1 output| + max|b2|
        c2[rb].yb.c = w2[rb]->b_abs;
        prog_add(c2[rb].yb, 1.0f, st[rb]);
        prog_add(c2[rb].yb, w2[rb]->g_abs, tr[rb]);
        c2[rb].y_amax = ra.amax();
        c2[rb].y_ash = !silu_on_load && b.RS[rb].h2 ? ra.ash() : nullptr;
      }
      RUN(run_conv_group(h, w2, c2, c.n_res, s));
      for (int rb = 0; rb < c.n_res; ++rb) {
        st[rb] = Rng{};
        st[rb].amax = c2[rb].y_amax;
        in1[rb] = Rng{c2[rb].y_ash, 0, c2[rb].y_amax, 0.f};
      }
    } else {  // last pair: ParallelBlock mean folded into the epilogues, in ResBlock order
      const ConvW* w2[NR];
      ConvCall cm[NR];
      for (int rb = 0; rb < c.n_res; ++rb) {
        ConvCall& cc = cm[rb];
        Act tin = b.Tb_in[rb];
        tin.r = tr[rb];
        cc = framed(tin, B, Lo, Co);
        cc.epi = dcx::EPI_RES;
        cc.res = b.R[rb];
        cc.macc = b.Mx;
        cc.mean = rb == 0 ? dcx::MEAN_FIRST : (rb == c.n_res - 1 ? dcx::MEAN_LAST : dcx::MEAN_MID);
        w2[rb] = &h->res[i][rb][ci][1];
        if (rb == c.n_res - 1) {
          // silu(mean): input of ups[i+1], or (fp32, in place) of conv_post
          if (b.last) cc.y2 = b.Mx;
          else cc.silu_to(b.next);  // input of the next ConvT
          // |mean| <= (1/3) sum over the ResBlocks of (max|state| + g2 max|c1 output| + max|b2|)
          float bc = 0.f;
          for (int m = 0; m < c.n_res; ++m) {
            const ConvW& wm = h->res[i][m][ci][1];
            bc += wm.b_abs / 3.0f;
            prog_add(cc.yb, 1.0f / 3.0f, st[m]);
            prog_add(cc.yb, wm.g_abs / 3.0f, tr[m]);
          }
          cc.yb.c = Builder::round_up((double)bc * (1.0 + 1e-6));
          cc.y_amax = b.next_amax;
          cc.y_ash = b.next_ash;
        }
      }
      // split-K mode: one grouped launch and one chained reduce; otherwise conv by conv (the
      // mean's order forbids the grouped unsplit kernel)
      int rc = 1;
      if (h->split_k >= 2 && c.n_res > 1) {
        ConvParams p[NR];
        double fl = 0, by = 0;
        for (int rb = 0; rb < c.n_res; ++rb) {
          RUN(conv_params(h, *w2[rb], cm[rb], false, p[rb]));
          fl += conv_flops(*w2[rb], cm[rb]);
          by += conv_bytes(*w2[rb], cm[rb]);
        }
        rc = run_conv_group_split(h, w2, cm, p, c.n_res, fl, by, s);
      }
      if (rc != 1) RUN(rc);
      else
        for (int rb = 0; rb < c.n_res; ++rb) RUN(run_conv(h, *w2[rb], cm[rb], s));
    }
  }
  if (!ra.ok()) return fail(h, DCX_ERR_STATE, "internal: h3 range slots exhausted");
  return DCX_OK;
}

// a tensor consumed by a small-Cout conv in fp32 (those kernels split while staging), range kept
Act fp32_form(dcx_codec* h, const Act& a, const ConvW& consumer) {
  if (!x6_mode(h) || !f32_input_ok(consumer)) return a;
  Act f{a.f ? a.f : reinterpret_cast<float*>(a.p), nullptr};
  f.r = a.r;
  return f;
}

int stage_generate(dcx_codec* h, CAct z, int B, int T, float* wav, Bump& ws, hipStream_t s) {
  const dcx_config& c = h->cfg;
  // z in conv_pre's h2 form, range-scaled by each clip's exact max (the fused pipeline's z as well)
  RUN(ensure_planes(h, z, (long long)B * T, c.vq_dim, ws, s, false, takes_h3_conv(h, h->conv_pre, T), B));
  const size_t per = (size_t)B * T * max_gen_width(c);
  // The ParallelBlock's ResBlocks are independent until the mean, so each keeps its own state and
  // the convs of one dilation index run as one grouped launch (run_conv_group).
  constexpr int NR = dcx::kMaxGroup;
  if (c.n_res > NR) return fail(h, DCX_ERR_INVALID_ARG, "more ResBlocks per stage than supported");
  if (2 + 36 * c.n_ups > RangeArena::kSlots) return fail(h, DCX_ERR_INVALID_ARG, "too many generator stages");
  float* X = ws.f(per);   // ConvT output (residual of each ResBlock's first pair)
  float* Mx = ws.f(per);  // ParallelBlock mean accumulator; silu(mean) of the last stage
  Act S = conv_input(h, ws, per);   // silu(stage input) -> ConvT
  Act XS = conv_input(h, ws, per);  // silu(X)
  float* R[NR];                     // ResBlock states
  Act RS[NR], Tb[NR];               // silu(R), silu(c1 output)
  for (int rb = 0; rb < c.n_res; ++rb) {
    R[rb] = ws.f(per);
    RS[rb] = conv_input(h, ws, per);
    Tb[rb] = conv_input(h, ws, per);
  }
  RangeArena ra;
  ra.reserve(ws, B);
  if (ws.dry) return DCX_OK;
  if (!ws.ok()) return fail(h, DCX_ERR_WORKSPACE, "workspace too small for generate");
  // the measured maxima only serve h3 consumers: none in the split-K latency mode or the fp32 mode,
  // where the epilogues then skip their range reductions and no slot is cleared (C5: one launch and
  // the reductions of ~40 epilogues per hop)
#ifndef DCX_DIAG_LAT_RANGES  // A/B build: the slots tracked in every mode (round-6 first form)
  if (!x6_mode(h) || h->split_k >= 2) ra.base = nullptr;
#endif
  if (ra.base) HIPCHK(h, dcx::launch_zero_words(ra.base, (long long)RangeArena::kSlots * B, s));
  // Tensors consumed by small-Cout convs are kept in fp32 (those kernels split them while
  // staging: the stages are bound by HBM traffic, and planes cost 6 B per element against 4).
  auto in_form = [&](const Act& a, const ConvW& consumer) -> Act { return fp32_form(h, a, consumer); };
  int C = c.gen_channels, L = T;
  {  // conv_pre, then the first stage's SiLU (generators.py:121,125) fused as the only output
    ConvCall cc = framed(z, B, T, c.vq_dim);
    Act S0 = S;
    S0.h2 = S.p && takes_h3_conv(h, h->ups[0], T);
    cc.silu_to(S0);
    cc.yb = prog_conv(h->conv_pre, z.r);
    cc.y_amax = ra.amax();
    cc.y_ash = S0.h2 ? ra.ash() : nullptr;
    RUN(run_conv(h, h->conv_pre, cc, s));
    S.r = Rng{cc.y_ash, 0, cc.y_amax, 0.f};
  }
  for (int i = 0; i < c.n_ups; ++i) {
    const ConvW& up = h->ups[i];
    const int Co = up.cout, Lo = L * c.up_rates[i];
    const ConvW& rconv = h->res[i][0][0][0];  // every ResBlock conv of the stage has Cin = Cout = Co
    Act S_i = in_form(S, up);
    S_i.h2 = S_i.p && takes_h3_conv(h, up, L);  // as conv_pre / the previous stage's mean epilogue wrote it
    Act XS_i = in_form(XS, rconv);
    Act RS_i[NR], Tb_i[NR];
    for (int rb = 0; rb < c.n_res; ++rb) {
      RS_i[rb] = in_form(RS[rb], rconv);
      Tb_i[rb] = in_form(Tb[rb], rconv);
    }
    // fp32-input stages: the first conv of each pair applies silu to X / R while staging, so
    // silu(X) and silu(R) are never written (7 activation tensors per stage less HBM traffic)
    const bool silu_on_load = x6_mode(h) && f32_input_ok(rconv);
    if (h3_stage(h, i, Lo)) {  // the ResBlock convs' inputs in the h2 layout (conv_gemm_x3dq)
      XS_i.h2 = true;
      for (int rb = 0; rb < c.n_res; ++rb) RS_i[rb].h2 = Tb_i[rb].h2 = true;
    }
    float* amax_X = ra.amax();
    {
      ConvCall cc = framed(S_i, B, L, C);
      cc.y = X;
      if (!silu_on_load) cc.silu_to(XS_i);
      cc.yb = prog_conv(up, S_i.r);
      cc.y_amax = amax_X;
      cc.y_ash = !silu_on_load && XS_i.h2 ? ra.ash() : nullptr;
      RUN(run_conv(h, up, cc, s));
      XS_i.r = Rng{cc.y_ash, 0, amax_X, 0.f};
    }
    PBlockBufs pb;
    pb.X = X;
    pb.XS = XS_i;
    for (int rb = 0; rb < c.n_res; ++rb) {
      pb.R[rb] = R[rb];
      pb.RS[rb] = RS_i[rb];
      pb.Tb[rb] = Tb[rb];
      pb.Tb_in[rb] = Tb_i[rb];
    }
    pb.Mx = Mx;
    pb.last = i == c.n_ups - 1;
    pb.amax_X = amax_X;
    pb.ra = &ra;
    if (!pb.last) {
      pb.next = in_form(S, h->ups[i + 1]);
      pb.next.h2 = pb.next.p && takes_h3_conv(h, h->ups[i + 1], Lo);
      pb.next_amax = ra.amax();
      pb.next_ash = pb.next.h2 ? ra.ash() : nullptr;
    }
    if (!ra.ok()) return fail(h, DCX_ERR_STATE, "internal: h3 range slots exhausted");
    RUN(run_parallel_block(h, i, B, Lo, pb, s));
    S.r = Rng{pb.next_ash, 0, pb.next_amax, 0.f};
    C = Co;
    L = Lo;
  }
  const bool bf = h->gemm_mode == DCX_GEMM_BF16;
  LAUNCH(h, s, "conv_post_tanh", 2.0 * B * L * C * c.gen_post_k, 4.0 * B * L * (C + 1),
         dcx::launch_conv_post_tanh(Mx, h->post_w, bf ? bf16_f(bf16_rne(h->post_b)) : h->post_b, wav, B, L, C,
                                    c.gen_post_k, bf ? 1 : 0, s));
  return DCX_OK;
}

// Marks a handle as inside a half-batch (stage_encode_decode): nested calls do not fork.
struct NoFork {
  dcx_codec* h;
  explicit NoFork(dcx_codec* h_) : h(h_) { h->no_fork = true; }
  ~NoFork() { h->no_fork = false; }
};

// conv_pre's input z of B clips x T frames: fp32, plus planes from the VQ up block's epilogue (x6)
// unless the generator splits z.f into h2 itself with each clip's exact range (launch_h2_ranged)
Act alloc_z(dcx_codec* h, Bump& ws, int B, int T) {
  const long long M = (long long)B * T;
  Act z;
  z.f = ws.f((size_t)M * h->cfg.vq_dim);
  if (x6_mode(h) && !(h->has_gen && takes_h3_conv(h, h->conv_pre, T))) z.p = ws.u16((size_t)M * h->cfg.vq_dim * 3);
  return z;
}

// mel -> encoder -> VQ encode -> VQ decode of B clips, into z (the generator's input)
int encode_clips_to_z(dcx_codec* h, const float* audio, int B, int64_t n, int32_t* codes, Act z, Bump& ws,
                      hipStream_t s) {
  const dcx_config& c = h->cfg;
  const int T = (int)frames_of(c, n);
  const long long M = (long long)B * T;
  Act mel = conv_input(h, ws, (size_t)M * c.n_mels);
  Act feat = conv_input(h, ws, (size_t)M * c.enc_dims[3]);
  feat.c1 = feat.p && takes_compact(h, h->vq_down, M);  // written by the encoder's final LayerNorm
  feat.h2 = feat.p && !feat.c1 && takes_h3(h, h->vq_down);  // h2 for the quantizer's down conv (x3dw)
  // (reserved whenever x6 mode could write it: a dry run sees no pointers, so sizes must not depend on them)
  if (x6_mode(h)) feat.row_ash = ws.i((size_t)M);
  if (feat.h2) feat.r.ash_row = feat.row_ash;  // scaled per row by the final LayerNorm (its exact row maxima)
  const size_t mark = ws.off;
  size_t need = mark;
  auto sub = [&](auto fn) -> int {  // each sub-stage reuses the tail of the workspace
    Bump tail(ws.base, ws.cap, ws.dry);
    tail.off = mark;
    int rc = fn(tail);
    need = std::max(need, tail.off);
    return rc;
  };
  if (!ws.dry && !ws.ok()) return fail(h, DCX_ERR_WORKSPACE, "workspace too small for encode_decode");
  RUN(sub([&](Bump& t) { return stage_mel(h, audio, B, n, mel, t, s); }));
  RUN(sub([&](Bump& t) { return stage_encode(h, CAct(mel), B, T, feat, t, s); }));
  RUN(sub([&](Bump& t) { return stage_vq_encode(h, CAct(feat), B, T, codes, nullptr, nullptr, nullptr, t, s); }));
  RUN(sub([&](Bump& t) { return stage_vq_decode(h, codes, B, T, z, nullptr, t, s); }));
  ws.off = need;
  return DCX_OK;
}

// a finalized handle without generator weights can never run the generator: its size is left out
// of the workspace (token extraction at C3's 256 clips would otherwise reserve 139 GB)
bool sizes_generator(const dcx_codec* h, const Bump& ws) { return !(ws.dry && h->finalized && !h->has_gen); }

int encode_decode_clips(dcx_codec* h, const float* audio, int B, int64_t n, int32_t* codes, float* wav, Bump& ws,
                        hipStream_t s) {
  const int T = (int)frames_of(h->cfg, n);
  Act z = alloc_z(h, ws, B, T);
  const size_t mark = ws.off;
  Bump front(ws.base, ws.cap, ws.dry);
  front.off = mark;
  RUN(encode_clips_to_z(h, audio, B, n, codes, z, front, s));
  size_t need = front.off;
  if (sizes_generator(h, ws)) {
    Bump tail(ws.base, ws.cap, ws.dry);
    tail.off = mark;
    RUN(stage_generate(h, CAct(z), B, T, wav, tail, s));
    need = std::max(need, tail.off);
  }
  if (ws.dry) ws.off = need;
  return DCX_OK;
}

// Half-batches on two streams (Knobs::enc_streams >= 2; 1 forks inside the encoder only): clips
// [0, B0) on the caller's stream and [B0, B) on the side stream, each in its own part of the
// workspace (half 0's, then half 1's: the sizes are linear in the clip count).  Every stage computes
// a clip alone (the reference's batch semantics: clips padded to one length, no cross-clip
// arithmetic), so the halves give the bits of the whole batch; the encoder then runs unforked inside
// each half.  2 (default): mel -> encoder -> VQ encode -> VQ decode per half, joined, then the
// generator on the whole batch, so the generator's long launches (the dominant kernel) run alone;
// 3: the generator per half too.  Not in the split-K latency mode, whose partial sums share one
// scratch region.
int stage_encode_decode(dcx_codec* h, const float* audio, int B, int64_t n, int32_t* codes, float* wav, Bump& ws,
                        hipStream_t s) {
  const int mode = h->knobs.enc_streams;
  if (B < 2 || mode < 2 || h->split_k >= 2 || (!ws.dry && !may_fork(h, s)) || h->no_fork)
    return encode_decode_clips(h, audio, B, n, codes, wav, ws, s);
  NoFork nf(h);
  const int B0 = (B + 1) / 2;
  const int T = (int)frames_of(h->cfg, n);
  const size_t start = ws.off;
  Act z;
  if (mode == 2) z = alloc_z(h, ws, B, T);
  const size_t mark = ws.off;
  // the halves' parts: [mark, e0) and [e0, e1) (sized by dry runs)
  auto half = [&](int b0, int nb, Bump& w, hipStream_t st) -> int {
    const bool dry = w.dry;
    const float* a = dry ? nullptr : audio + (long long)b0 * n;
    int32_t* cd = dry ? nullptr : codes + (long long)b0 * T;
    if (mode == 2) return encode_clips_to_z(h, a, nb, n, cd, act_rows_out(z, b0, (long long)b0 * T, h->cfg.vq_dim), w, st);
    return encode_decode_clips(h, a, nb, n, cd, dry ? nullptr : wav + (long long)b0 * T * h->cfg.hop, w, st);
  };
  Bump d0(nullptr, 0, true);
  d0.off = mark;
  RUN(half(0, B0, d0, s));
  Bump d1(nullptr, 0, true);
  d1.off = d0.off;
  RUN(half(B0, B - B0, d1, s));
  size_t need = d1.off;
  if (mode == 2 && sizes_generator(h, ws)) {
    Bump dg(nullptr, 0, true);
    dg.off = mark;
    RUN(stage_generate(h, CAct(z), B, T, nullptr, dg, s));
    need = std::max(need, dg.off);
  }
  if (ws.dry) {  // sized for the one-stream plan too (a call captured into a hipGraph does not fork)
    Bump one(nullptr, 0, true);
    one.off = start;
    RUN(encode_decode_clips(h, nullptr, B, n, nullptr, nullptr, one, s));
    ws.off = std::max(need, one.off);
    return DCX_OK;
  }
  if (need > ws.cap) return fail(h, DCX_ERR_WORKSPACE, "workspace too small for encode_decode");
  Bump w0(ws.base, ws.cap, false), w1(ws.base, ws.cap, false);
  w0.off = mark;
  w1.off = d0.off;
  HIPCHK(h, hipEventRecord(h->fork_ev, s));
  HIPCHK(h, hipStreamWaitEvent(h->side, h->fork_ev, 0));
  const int rc0 = half(0, B0, w0, s);
  const int rc1 = rc0 != DCX_OK ? rc0 : half(B0, B - B0, w1, h->side);
  // joined whatever happened, so the caller's stream never runs ahead of the side stream's work
  const hipError_t e0 = hipEventRecord(h->join_ev, h->side);
  const hipError_t e1 = hipStreamWaitEvent(s, h->join_ev, 0);
  RUN(rc1);
  HIPCHK(h, e0);
  HIPCHK(h, e1);
  if (mode == 2) {
    Bump tail(ws.base, ws.cap, false);
    tail.off = mark;
    RUN(stage_generate(h, CAct(z), B, T, wav, tail, s));
  }
  return DCX_OK;
}

// ---------------- single reference modules (dcx_module_forward) ----------------
// "<prefix>.%d[.%d]" matched exactly (the whole name consumed).
bool match_idx(const std::string& m, const char* fmt, int* a, int* b = nullptr) {
  int n = -1;
  const int want = b ? 2 : 1;
  const int got = b ? std::sscanf(m.c_str(), fmt, a, b, &n) : std::sscanf(m.c_str(), fmt, a, &n);
  return got == want && n == (int)m.size();
}

// Input / output widths of a module (dcx_module_io): cin, cout (0: int32 codes), output rows per
// input row.  False for unknown names.
bool module_io(const dcx_codec* h, const std::string& m, int& cin, int& cout, int& rate) {
  const dcx_config& c = h->cfg;
  int a = -1, b = -1;
  rate = 1;
  auto set = [&](int i, int o) {
    cin = i;
    cout = o;
    return true;
  };
  if (match_idx(m, "encoder.stages.%d.%d%n", &a, &b) && a >= 0 && a < 4 && b >= 0 && b < c.enc_depths[a])
    return set(c.enc_dims[a], c.enc_dims[a]);
  if (m == "encoder.downsample_layers.0") return set(c.n_mels, c.enc_dims[0]);
  if (m == "encoder.downsample_layers.0.1") return set(c.enc_dims[0], c.enc_dims[0]);
  if (match_idx(m, "encoder.downsample_layers.%d%n", &a) && a >= 1 && a < 4) return set(c.enc_dims[a - 1], c.enc_dims[a]);
  if (match_idx(m, "encoder.downsample_layers.%d.0%n", &a) && a >= 1 && a < 4) return set(c.enc_dims[a - 1], c.enc_dims[a - 1]);
  if (m == "encoder.norm") return set(c.enc_dims[3], c.enc_dims[3]);
  if (m == "quantizer.downsample.0" || m == "quantizer.downsample.0.1" || m == "quantizer.upsample.0" ||
      m == "quantizer.upsample.0.1")
    return set(c.vq_dim, c.vq_dim);
  if (m == "quantizer.grvq.rvqs.0.project_in") return set(c.vq_dim, c.codebook_dim);
  if (m == "quantizer.search") return set(c.codebook_dim, 0);
  if (m == "generator.conv_pre") return set(c.vq_dim, c.gen_channels);
  int ch = c.gen_channels;
  for (int i = 0; i < c.n_ups; ++i) {
    if (m == "generator.ups." + std::to_string(i)) {
      rate = c.up_rates[i];
      return set(ch, ch / 2);
    }
    ch /= 2;
    if (match_idx(m, "generator.resblocks.%d.blocks.%d%n", &a, &b) && a == i && b >= 0 && b < c.n_res) return set(ch, ch);
    if (match_idx(m, "generator.resblocks.%d%n", &a) && a == i) return set(ch, ch);
  }
  if (m == "generator.conv_post") return set(ch, 1);
  return false;
}

// One module of the reference by its state-dict prefix, on the handle's packed weights and through
// the same launches the stages use.  x / y: channels-last fp32 [B][L][C] (codes int32 [B][L] for
// "quantizer.search").  See dcx_module_forward in the header for the list.
int stage_module(dcx_codec* h, const std::string& m, const float* x, int B, int L, void* yv, Bump& ws, hipStream_t s) {
  const dcx_config& c = h->cfg;
  const long long M = (long long)B * L;
  float* y = static_cast<float*>(yv);
  int a = -1, b = -1;
  // Sequential stems of the encoder (encoders.py:22-39): conv k7 + channels-first LayerNorm (i = 0),
  // LayerNorm + 1x1 conv (i >= 1)
  if (m == "encoder.downsample_layers.0") {
    CAct in(x, nullptr);
    RUN(ensure_planes(h, in, M, c.n_mels, ws, s));
    float* t = ws.f((size_t)M * c.enc_dims[0]);
    if (ws.dry) return DCX_OK;
    if (!ws.ok()) return fail(h, DCX_ERR_WORKSPACE, "workspace too small for the module");
    ConvCall cc = framed(in, B, L, c.n_mels);
    cc.y = t;
    RUN(run_conv(h, h->stem, cc, s));
    return run_ln(h, h->stem_ln, t, Act{y, nullptr}, M, s, /*bf16_in=*/true);
  }
  if (match_idx(m, "encoder.downsample_layers.%d%n", &a) && a >= 1 && a < 4) {
    Act ln = conv_input(h, ws, (size_t)M * c.enc_dims[a - 1]);
    if (x6_mode(h)) ln.row_ash = ws.i((size_t)M);
    if (ws.dry) return DCX_OK;
    if (!ws.ok()) return fail(h, DCX_ERR_WORKSPACE, "workspace too small for the module");
    ln.c1 = ln.p && takes_compact(h, h->ds_conv[a], M);
    ln.h2 = ln.p && ln.row_ash && takes_h3(h, h->ds_conv[a]);
    ln.r.ash_row = ln.h2 ? ln.row_ash : nullptr;
    RUN(run_ln(h, h->ds_ln[a], x, ln, M, s));
    ConvCall cd = pointwise(ln, M);
    cd.y = y;
    return run_conv(h, h->ds_conv[a], cd, s);
  }
  // the quantizer's down / up paths (grfvq.py:68-96): conv (k = factor) or ConvT, then a ConvNeXtBlock
  if (m == "quantizer.downsample.0" || m == "quantizer.upsample.0") {
    const bool down = m == "quantizer.downsample.0";
    const int D = c.vq_dim;
    CAct in(x, nullptr);
    // the down conv in h3 as in the pipeline (range floor: the encoder's final LayerNorm bound)
    RUN(ensure_planes(h, in, M, D, ws, s, false, down && takes_h3(h, h->vq_down), 0));
    Act ln = conv_input(h, ws, (size_t)M * D);
    Act hid = conv_input(h, ws, (size_t)M * 4 * D);
    row_ranges(h, ws, M, ln, hid);
    if (ws.dry) return DCX_OK;
    if (!ws.ok()) return fail(h, DCX_ERR_WORKSPACE, "workspace too small for the module");
    ConvCall cc = pointwise(in, M);
    cc.y = y;
    RUN(run_conv(h, down ? h->vq_down : h->vq_up, cc, s));
    return run_block(h, down ? h->vq_down_blk : h->vq_up_blk, y, nullptr, B, L, ln, hid, s);
  }
  if (m == "quantizer.grvq.rvqs.0.project_in") {  // residual_vq.py:152
    CAct in(x, nullptr);
    RUN(ensure_planes(h, in, M, c.vq_dim, ws, s, false, takes_h3(h, h->vq_pin), 0));
    if (ws.dry) return DCX_OK;
    if (!ws.ok()) return fail(h, DCX_ERR_WORKSPACE, "workspace too small for the module");
    ConvCall cp = pointwise(in, M);
    cp.y = y;
    return run_conv(h, h->vq_pin, cp, s);
  }
  // ConvNeXtBlock (convnext_utils.py:263-282)
  const BlockW* blk = nullptr;
  if (match_idx(m, "encoder.stages.%d.%d%n", &a, &b) && a >= 0 && a < 4 && b >= 0 && b < (int)h->blocks[a].size())
    blk = &h->blocks[a][b];
  else if (m == "quantizer.downsample.0.1") blk = &h->vq_down_blk;
  else if (m == "quantizer.upsample.0.1") blk = &h->vq_up_blk;
  if (blk) {
    if (!blk->C) return fail(h, DCX_ERR_STATE, "module weights not finalized");
    Act ln = conv_input(h, ws, (size_t)M * blk->C);
    Act hid = conv_input(h, ws, (size_t)M * 4 * blk->C);
    row_ranges(h, ws, M, ln, hid);
    if (ws.dry) return DCX_OK;
    if (!ws.ok()) return fail(h, DCX_ERR_WORKSPACE, "workspace too small for the module");
    HIPCHK(h, hipMemcpyAsync(y, x, sizeof(float) * M * blk->C, hipMemcpyDeviceToDevice, s));
    return run_block(h, *blk, y, nullptr, B, L, ln, hid, s);
  }
  // channels-first LayerNorm (convnext_utils.py:186-213)
  const LnW* lw = nullptr;
  if (m == "encoder.downsample_layers.0.1") lw = &h->stem_ln;
  else if (match_idx(m, "encoder.downsample_layers.%d.0%n", &a) && a >= 1 && a < 4) lw = &h->ds_ln[a];
  else if (m == "encoder.norm") lw = &h->enc_norm;
  if (lw) {
    if (ws.dry) return DCX_OK;
    return run_ln(h, *lw, x, Act{y, nullptr}, M, s);
  }
  // nearest-code search on x_pjt_in (EuclideanCodebook.forward, vector_quantize_pytorch.py:496-506)
  if (m == "quantizer.search") {
    if (!h->codebook) return fail(h, DCX_ERR_STATE, "module weights not finalized");
    const int CD = c.codebook_dim, NC = c.codebook_size;
    // bf16 mode: the pipeline's search (compact bf16 x_pjt_in for the one-product prefilter, exact fp64
    // rescore of x as given).  The reference searches x.float() with autocast off
    // (vector_quantize_pytorch.py:462-498), x being project_in's bf16 output; row_sqnorm's |x - bf16(x)|^2
    // keeps the prefilter's bound valid for an input that is not bf16-valued.
    const bool x6 = x6_mode(h);
    const int xl = vq_xlayout(h, M);
    const int ntiles = x6 ? dcx::vq_prefilter_ntiles(NC, CD, M, xl) : dcx::vq_argmin_ntiles(NC);
    unsigned short* P6 = x6 ? ws.u16((size_t)M * CD * 3) : nullptr;
    const VqScratch vs = vq_scratch(h, ws, M, ntiles, x6);
    if (ws.dry) return DCX_OK;
    if (!ws.ok()) return fail(h, DCX_ERR_WORKSPACE, "workspace too small for the module");
    if (x6) LAUNCH(h, s, "split_planes", 0, 10.0 * M * CD, dcx::launch_split_planes(x, P6, M, CD, xl, s));
    return run_vq_search(h, x, P6, xl, M, vs, ntiles, static_cast<int32_t*>(yv), s);
  }
  if (!h->has_gen && m.rfind("generator.", 0) == 0) return fail(h, DCX_ERR_STATE, "generator weights were not finalized");
  if (m == "generator.conv_pre") {  // generators.py:121
    CAct in(x, nullptr);
    RUN(ensure_planes(h, in, M, c.vq_dim, ws, s, false, takes_h3_conv(h, h->conv_pre, L), B));
    if (ws.dry) return DCX_OK;
    if (!ws.ok()) return fail(h, DCX_ERR_WORKSPACE, "workspace too small for the module");
    ConvCall cc = framed(in, B, L, c.vq_dim);
    cc.y = y;
    return run_conv(h, h->conv_pre, cc, s);
  }
  if (m == "generator.conv_post") {  // generators.py:141-145: activation_post (SiLU), conv_post, tanh
    int ch = c.gen_channels;
    for (int i = 0; i < c.n_ups; ++i) ch /= 2;
    float* t = ws.f((size_t)M * ch);
    if (ws.dry) return DCX_OK;
    if (!ws.ok()) return fail(h, DCX_ERR_WORKSPACE, "workspace too small for the module");
    LAUNCH(h, s, "silu_act", 0, 8.0 * M * ch, dcx::launch_silu_act(x, t, nullptr, M, ch, s));
    const bool bf = h->gemm_mode == DCX_GEMM_BF16;
    LAUNCH(h, s, "conv_post_tanh", 2.0 * M * ch * c.gen_post_k, 4.0 * M * (ch + 1),
           dcx::launch_conv_post_tanh(t, h->post_w, bf ? bf16_f(bf16_rne(h->post_b)) : h->post_b, y, B, L, ch,
                                      c.gen_post_k, bf ? 1 : 0, s));
    return DCX_OK;
  }
  // ConvTranspose1d (generators.py:118-147, ups[i])
  if (match_idx(m, "generator.ups.%d%n", &a) && a >= 0 && a < c.n_ups) {
    const ConvW& up = h->ups[a];
    CAct in(x, nullptr);
    if (!(x6_mode(h) && f32_input_ok(up))) RUN(ensure_planes(h, in, M, up.cin, ws, s, false, takes_h3_conv(h, up, L), B));
    if (ws.dry) return DCX_OK;
    if (!ws.ok()) return fail(h, DCX_ERR_WORKSPACE, "workspace too small for the module");
    ConvCall cc = framed(in, B, L, up.cin);
    cc.y = y;
    return run_conv(h, up, cc, s);
  }
  auto in_form = [&](const Act& v, const ConvW& consumer) -> Act { return fp32_form(h, v, consumer); };
  // ResBlock1 (convnext_utils.py:106-113), as per-conv launches of the production conv kernels
  if (match_idx(m, "generator.resblocks.%d.blocks.%d%n", &a, &b) && a >= 0 && a < c.n_ups && b >= 0 && b < c.n_res) {
    const ConvW& w0 = h->res[a][b][0][0];
    const int C = w0.cout;
    Act XS = conv_input(h, ws, (size_t)M * C);  // silu(state), the c1 input (unless silu on load)
    Act Tb = conv_input(h, ws, (size_t)M * C);  // silu(c1 output)
    RangeArena ra;
    ra.reserve(ws, B);
    if (ws.dry) return DCX_OK;
    if (!ws.ok()) return fail(h, DCX_ERR_WORKSPACE, "workspace too small for the module");
    HIPCHK(h, dcx::launch_zero_words(ra.base, (long long)RangeArena::kSlots * B, s));
    const bool silu_on_load = x6_mode(h) && f32_input_ok(w0);
    Act XSi = in_form(XS, w0), Tbi = in_form(Tb, w0);
    XSi.h2 = Tbi.h2 = h3_stage(h, a, L);
    HIPCHK(h, hipMemcpyAsync(y, x, sizeof(float) * M * C, hipMemcpyDeviceToDevice, s));
    Rng st;  // the state's range: its measured max |.| (and, in h2, its silu's shift)
    st.amax = ra.amax();
    if (!silu_on_load && XSi.h2) {
      int* sh = ra.ash();
      LAUNCH(h, s, "h2_ranged", 0, 12.0 * M * C,
             dcx::launch_h2_ranged(y, nullptr, XSi.p, B, L, C, 1, 0.f, const_cast<float*>(st.amax), sh, h->rflag, s));
      st.ash = sh;
    } else {
      LAUNCH(h, s, "clip_amax", 0, 4.0 * M * C, dcx::launch_clip_amax(y, B, L, C, const_cast<float*>(st.amax), s));
      if (!silu_on_load)
        LAUNCH(h, s, "silu_act", 0, 10.0 * M * C, dcx::launch_silu_act(y, XSi.f, XSi.p, M, C, s, 0));
    }
    for (int ci = 0; ci < 3; ++ci) {
      const ConvW& w1 = h->res[a][b][ci][0];
      const ConvW& w2 = h->res[a][b][ci][1];
      Act in1 = silu_on_load ? Act{y, nullptr} : XSi;
      in1.r = st;
      ConvCall c1 = framed(in1, B, L, C);
      c1.silu_in = silu_on_load;
      c1.silu_to(Tbi);
      c1.yb = prog_conv(w1, st);
      c1.y_amax = ra.amax();
      c1.y_ash = Tbi.h2 ? ra.ash() : nullptr;
      RUN(run_conv(h, w1, c1, s));
      const Rng tr{c1.y_ash, 0, c1.y_amax, 0.f};
      Act tin = Tbi;
      tin.r = tr;
      ConvCall c2 = framed(tin, B, L, C);
      c2.epi = dcx::EPI_RES;
      c2.res = y;
      c2.y = y;
      if (!silu_on_load && ci < 2) c2.silu_to(XSi);
      c2.yb.c = w2.b_abs;  // |state + c2 + b2| <= max|state| + g2 max|c1 output| + max|b2|
      prog_add(c2.yb, 1.0f, Rng{nullptr, 0, st.amax, 0.f});
      prog_add(c2.yb, w2.g_abs, tr);
      c2.y_amax = ra.amax();
      c2.y_ash = !silu_on_load && ci < 2 && XSi.h2 ? ra.ash() : nullptr;
      RUN(run_conv(h, w2, c2, s));
      st = Rng{c2.y_ash, 0, c2.y_amax, 0.f};
    }
    return DCX_OK;
  }
  // ParralelBlock of stage i followed by the generator's SiLU: silu(mean of the ResBlock1s), fp32
  if (match_idx(m, "generator.resblocks.%d%n", &a) && a >= 0 && a < c.n_ups) {
    constexpr int NR = dcx::kMaxGroup;
    const ConvW& w0 = h->res[a][0][0][0];
    const int C = w0.cout;
    const size_t per = (size_t)M * C;
    float* X = ws.f(per);
    Act XS = conv_input(h, ws, per);
    PBlockBufs pb;
    Act RS[NR];
    for (int rb = 0; rb < c.n_res; ++rb) {
      pb.R[rb] = ws.f(per);
      RS[rb] = conv_input(h, ws, per);
      pb.Tb[rb] = conv_input(h, ws, per);
    }
    RangeArena ra;
    ra.reserve(ws, B);
    if (ws.dry) return DCX_OK;
    if (!ws.ok()) return fail(h, DCX_ERR_WORKSPACE, "workspace too small for the module");
    HIPCHK(h, dcx::launch_zero_words(ra.base, (long long)RangeArena::kSlots * B, s));
    const bool silu_on_load = x6_mode(h) && f32_input_ok(w0);
    HIPCHK(h, hipMemcpyAsync(X, x, sizeof(float) * per, hipMemcpyDeviceToDevice, s));
    pb.X = X;
    const bool h3 = h3_stage(h, a, L);
    pb.XS = in_form(XS, w0);
    pb.XS.h2 = h3;
    for (int rb = 0; rb < c.n_res; ++rb) {
      pb.RS[rb] = in_form(RS[rb], w0);
      pb.Tb_in[rb] = in_form(pb.Tb[rb], w0);
      pb.RS[rb].h2 = pb.Tb_in[rb].h2 = h3;
    }
    float* amax_X = ra.amax();
    if (!silu_on_load && h3) {
      int* sh = ra.ash();
      LAUNCH(h, s, "h2_ranged", 0, 12.0 * per,
             dcx::launch_h2_ranged(X, nullptr, pb.XS.p, B, L, C, 1, 0.f, amax_X, sh, h->rflag, s));
      pb.XS.r = Rng{sh, 0, amax_X, 0.f};
    } else {
      LAUNCH(h, s, "clip_amax", 0, 4.0 * per, dcx::launch_clip_amax(X, B, L, C, amax_X, s));
      if (!silu_on_load)
        LAUNCH(h, s, "silu_act", 0, 10.0 * per, dcx::launch_silu_act(X, pb.XS.f, pb.XS.p, M, C, s, 0));
    }
    pb.Mx = y;
    pb.last = true;
    pb.amax_X = amax_X;
    pb.ra = &ra;
    return run_parallel_block(h, a, B, L, pb, s);
  }
  return fail(h, DCX_ERR_INVALID_ARG, "unknown module: " + m);
}

int check_ready(dcx_codec* h, bool need_gen) {
  if (!h) return DCX_ERR_INVALID_ARG;
  if (!h->finalized) return fail(h, DCX_ERR_STATE, "dcx_finalize has not been called");
  if (need_gen && !h->has_gen) return fail(h, DCX_ERR_STATE, "generator weights were not finalized");
  int dev = -1;
  hipGetDevice(&dev);
  if (dev != h->device) return fail(h, DCX_ERR_STATE, "handle belongs to another HIP device");
  return DCX_OK;
}

}  // namespace

// =========================================================================================
// C ABI
// =========================================================================================
extern "C" {

int dcx_abi_version(void) { return DCX_ABI_VERSION; }

#ifndef DCX_BUILD_ID
#define DCX_BUILD_ID "unversioned"
#endif
const char* dcx_build_id(void) { return DCX_BUILD_ID; }

const char* dcx_status_string(int st) {
  switch (st) {
    case DCX_OK: return "ok";
    case DCX_ERR_INVALID_ARG: return "invalid argument";
    case DCX_ERR_MISSING_WEIGHT: return "missing weight";
    case DCX_ERR_STATE: return "invalid state";
    case DCX_ERR_HIP: return "HIP error";
    case DCX_ERR_OOM: return "out of device memory";
    case DCX_ERR_WORKSPACE: return "workspace too small";
    case DCX_ERR_UNSUPPORTED: return "unsupported input format";
    default: return "unknown status";
  }
}

void dcx_default_config(dcx_config* c) {
  std::memset(c, 0, sizeof(*c));
  c->sample_rate = 24000;
  c->n_fft = 1024; c->hop = 256; c->win = 1024; c->n_mels = 128;
  c->f_min = 0.f; c->f_max = 12000.f;
  const int dep[4] = {3, 3, 9, 3}, dim[4] = {256, 512, 768, 1024};
  for (int i = 0; i < 4; ++i) { c->enc_depths[i] = dep[i]; c->enc_dims[i] = dim[i]; }
  c->vq_dim = 1024; c->codebook_dim = 3584; c->codebook_size = 32768;
  c->gen_channels = 1024; c->gen_pre_k = 13; c->gen_post_k = 13;
  c->n_ups = 5;
  const int ur[5] = {8, 4, 2, 2, 2}, uk[5] = {16, 12, 4, 4, 4};
  for (int i = 0; i < 5; ++i) { c->up_rates[i] = ur[i]; c->up_kernels[i] = uk[i]; }
  c->n_res = 3;
  const int rk[3] = {3, 7, 11};
  for (int i = 0; i < 3; ++i) {
    c->res_kernels[i] = rk[i];
    c->res_dilations[i][0] = 1; c->res_dilations[i][1] = 3; c->res_dilations[i][2] = 5;
  }
}

const char* dcx_last_error(const dcx_codec* h) { return h ? h->err.c_str() : "null handle"; }

int dcx_create(const dcx_config* cfg, dcx_codec** out) {
  if (!cfg || !out) return DCX_ERR_INVALID_ARG;
  *out = nullptr;
  const dcx_config& c = *cfg;
  bool ok = c.n_fft == 1024 && c.win == 1024 && c.hop == 256 && c.n_mels % 16 == 0 && c.n_mels > 0 &&
            c.vq_dim == c.enc_dims[3] && c.codebook_dim % 16 == 0 && c.codebook_size % 128 == 0 &&
            c.n_ups >= 1 && c.n_ups <= 8 && c.n_res == 3 && c.gen_pre_k % 2 == 1 && c.gen_post_k % 2 == 1;
  for (int i = 0; i < 4 && ok; ++i) ok = c.enc_dims[i] % 256 == 0 && c.enc_dims[i] <= 1024 && c.enc_depths[i] >= 0;
  int ch = c.gen_channels;
  for (int i = 0; i < c.n_ups && ok; ++i) {
    ok = c.up_rates[i] >= 1 && c.up_rates[i] <= dcx::kMaxPhases && c.up_kernels[i] % c.up_rates[i] == 0 &&
         (c.up_kernels[i] - c.up_rates[i]) % 2 == 0;
    ch /= 2;
    ok = ok && ch % 32 == 0;
  }
  ok = ok && (ch == 32 || ch == 64);
  for (int i = 0; i < 3 && ok; ++i) ok = c.res_kernels[i] % 2 == 1;
  if (!ok) return DCX_ERR_INVALID_ARG;
  auto h = new (std::nothrow) dcx_codec();
  if (!h) return DCX_ERR_OOM;
  h->cfg = c;
  hipGetDevice(&h->device);
  const char* nrp = std::getenv("DCX_NO_RESPAIR");
  h->res_pair = !(nrp && nrp[0] == '1');
  const char* ncp = std::getenv("DCX_NO_COMPACT");
  h->compact = !(ncp && ncp[0] == '1');
  const char* vpr = std::getenv("DCX_VQ_PAIRS_PER_ROW");
  if (vpr && vpr[0]) h->vq_pairs_per_row = std::max(0, std::atoi(vpr));
  knobs_from_env(h->knobs);
  *out = h;
  return DCX_OK;
}

void dcx_destroy(dcx_codec* h) {
  if (!h) return;
  for (void* p : h->allocs) hipFree(p);
  for (auto e : h->events) hipEventDestroy(e);
  if (h->fork_ev) hipEventDestroy(h->fork_ev);
  if (h->join_ev) hipEventDestroy(h->join_ev);
  if (h->side) hipStreamDestroy(h->side);
  delete h;
}

int dcx_set_tensor(dcx_codec* h, const char* name, const float* data, int32_t ndim, const int64_t* shape) {
  if (!h || !name || (!data && ndim > 0) || ndim < 0 || ndim > 8) return fail(h, DCX_ERR_INVALID_ARG, "bad tensor");
  if (h->finalized) return fail(h, DCX_ERR_STATE, "dcx_set_tensor after dcx_finalize");
  HostTensor t;
  t.shape.assign(shape, shape + ndim);
  const int64_t n = t.numel();
  if (n < 0) return fail(h, DCX_ERR_INVALID_ARG, "negative shape");
  t.data.assign(data, data + n);
  h->host[name] = std::move(t);
  return DCX_OK;
}

static int build_all(dcx_codec* h, Builder& B, int32_t with_generator) {
  const dcx_config& c = h->cfg;
  // ---- mel front end: DFT basis as a 4-tap conv over 256-sample rows ------------------
  {
    const int N = c.n_fft, nb = N / 2 + 1;
    std::vector<double> win(N);
    for (int n = 0; n < N; ++n) win[n] = 0.5 - 0.5 * std::cos(2.0 * M_PI * n / N);  // hann, periodic
    std::vector<float> basis((size_t)N * N, 0.f);  // [col][n]; cols: re 0..512, im 1..511
    for (int k = 0; k < nb; ++k)
      for (int n = 0; n < N; ++n) {
        const long long kn = ((long long)k * n) % N;
        basis[(size_t)k * N + n] = (float)(win[n] * std::cos(2.0 * M_PI * kn / N));
        if (k > 0 && k < nb - 1) basis[(size_t)(nb + k - 1) * N + n] = (float)(-win[n] * std::sin(2.0 * M_PI * kn / N));
      }
    h->dft.cin = c.hop; h->dft.cout = N; h->dft.taps = N / c.hop; h->dft.in_step = 1;
    h->dft.w = B.upload(basis);
    h->dft.w6 = B.split_pack(basis, 1, N, N / c.hop, c.hop);
    const int kpad = (nb + 31) / 32 * 32;  // even number of 16-deep chunks (x6 kernels step in pairs)
    std::vector<double> fb = mel_fb(nb, c.f_min, c.f_max, c.n_mels, c.sample_rate);
    std::vector<float> pk((size_t)c.n_mels * kpad, 0.f);
    for (int m = 0; m < c.n_mels; ++m)
      for (int k = 0; k < nb; ++k) pk[(size_t)m * kpad + k] = (float)fb[(size_t)k * c.n_mels + m];
    h->melfb.cin = kpad; h->melfb.cout = c.n_mels; h->melfb.taps = 1;
    h->melfb.w = B.upload(pk);
    h->melfb.w6 = B.split_pack(pk, 1, c.n_mels, 1, kpad);
  }
  // ---- encoder --------------------------------------------------------------------------
  {
    const std::string e = "encoder.";
    h->stem = B.conv(e + "downsample_layers.0.0", c.n_mels, c.enc_dims[0], 7, 1, 3);
    h->stem_ln = B.ln(e + "downsample_layers.0.1", c.enc_dims[0]);
    for (int i = 0; i < 4; ++i) {
      if (i > 0) {
        const std::string p = e + "downsample_layers." + std::to_string(i);
        h->ds_ln[i] = B.ln(p + ".0", c.enc_dims[i - 1]);
        h->ds_conv[i] = B.conv(p + ".1", c.enc_dims[i - 1], c.enc_dims[i], 1, 1, 0, true, true);  // + h3 weights
      }
      h->blocks[i].clear();
      for (int j = 0; j < c.enc_depths[i]; ++j)
        h->blocks[i].push_back(B.block(e + "stages." + std::to_string(i) + "." + std::to_string(j), c.enc_dims[i]));
    }
    h->enc_norm = B.ln(e + "norm", c.enc_dims[3]);
  }
  // ---- quantizer ------------------------------------------------------------------------
  {
    const std::string q = "quantizer.";
    const int D = c.vq_dim, CD = c.codebook_dim, NC = c.codebook_size;
    h->vq_down = B.conv(q + "downsample.0.0", D, D, 1, 1, 0, true, true);  // + h3 weights
    h->vq_down_blk = B.block(q + "downsample.0.1", D);
    h->vq_up = B.convT(q + "upsample.0.0", D, D, 1, 1);
    h->vq_up_blk = B.block(q + "upsample.0.1", D);
    h->vq_pin = B.conv(q + "grvq.rvqs.0.project_in", D, CD, 1, 1, 0, true, true);  // + h3 weights
    ConvW pout = B.conv(q + "grvq.rvqs.0.project_out", CD, D, 1, 1, 0);
    auto emb = B.need(q + "grvq.rvqs.0.layers.0._codebook.embed", {1, NC, CD});
    if (emb) {
      std::vector<float> e2(NC);
      std::vector<double> e2d(NC);
      double e2m = 0;
      for (int i = 0; i < NC; ++i) {
        double sacc = 0;
        for (int d = 0; d < CD; ++d) sacc += (double)emb->data[(size_t)i * CD + d] * emb->data[(size_t)i * CD + d];
        e2[i] = (float)sacc;
        e2d[i] = sacc;
        e2m = std::max(e2m, sacc);
      }
      h->e2d = (double*)B.upload_raw(e2d.data(), e2d.size() * sizeof(double));
      // rounded up so the prefilter bound stays an upper bound
      h->e2max = std::nextafter((float)e2m, INFINITY);
      h->emax = std::nextafter((float)std::sqrt(e2m), INFINITY);
      h->vq_stats = (int*)B.upload(std::vector<float>(2, 0.f));  // zero counters
      h->codebook = B.upload(emb->data);
      h->codebook6 = B.split_pack(emb->data, 1, NC, 1, CD);
      h->e2 = B.upload(e2);
      // max |e - bf16(e)| in fp64, rounded up (vq_prefilter_b1's bound)
      double d2m = 0;
      for (int i = 0; i < NC; ++i) {
        double sacc = 0;
        for (int d = 0; d < CD; ++d) {
          const float v = emb->data[(size_t)i * CD + d];
          const double r = (double)v - (double)bf16_f(bf16_rne(v));
          sacc += r * r;
        }
        d2m = std::max(d2m, sacc);
      }
      h->dmax = std::nextafter((float)(std::sqrt(d2m) * (1.0 + 1e-12)), INFINITY);
      if (dcx::vq_b1_takes(NC, CD)) h->codebook_b1 = B.compact_pack(emb->data, NC, CD);
#ifdef DCX_VQ_OLD
      if (dcx::vq_bk_takes(NC, CD)) {
        h->codebook_bk = (unsigned short*)B.alloc((size_t)NC * CD);  // NC * CD * 2 bf16 (hi, mid)
        if (!B.bad() && !B.dry &&
            (dcx::launch_repack_codebook_bk(h->codebook6, NC, CD, h->codebook_bk, 0) != hipSuccess ||
             hipDeviceSynchronize() != hipSuccess))
          return fail(h, DCX_ERR_HIP, "bf16 codebook repack failed");
      }
#endif
    }
    // decode table: project_out applied to every code once, E * W_out^T + b_out.  Row NC holds
    // project_out(0) = b_out, the row of the reference's masked code -1 (residual_vq.py:120-127:
    // masked_fill(-1 -> 0), gather, then the gathered vector zeroed before project_out).
    h->ptable = B.alloc((size_t)(NC + 1) * D);
    h->ptable6 = (unsigned short*)B.alloc((size_t)(NC + 1) * D * 3 / 2);
    if (!B.bad() && !B.dry) {
      // built once with the fp32 MFMA path (the codebook is not held as activation planes)
      ConvCall cp = pointwise(CAct(h->codebook, nullptr), NC);
      cp.y = h->ptable;
      int rc = run_conv(h, pout, cp, 0, /*force_f32=*/true);
      if (rc != DCX_OK) return rc;
      if (hipMemcpy(h->ptable + (size_t)NC * D, pout.b, sizeof(float) * D, hipMemcpyDeviceToDevice) != hipSuccess ||
          dcx::launch_split_planes(h->ptable, h->ptable6, NC + 1, D, 0, 0) != hipSuccess ||
          hipDeviceSynchronize() != hipSuccess)
        return fail(h, DCX_ERR_HIP, "decode-table build failed");
    }
    // The bf16 mode's table: project_out under the reference's autocast (residual_vq.py:138 inside
    // distil_codec.py:590), bf16(bf16(E) W_out16^T + b_out16) by the one-product conv on the codebook
    // as activation planes (scratch); row NC = bf16(b_out) (the masked code).  Built in a scratch fp32
    // table, then split.
    h->ptable6b = (unsigned short*)B.alloc((size_t)(NC + 1) * D * 3 / 2);
    if (!B.bad() && !B.dry && h->codebook) {
      float* tmp = nullptr;
      unsigned short* e6 = nullptr;
      if (hipMalloc(&tmp, sizeof(float) * (size_t)(NC + 1) * D) != hipSuccess) return fail(h, DCX_ERR_OOM, "hipMalloc failed");
      if (hipMalloc(&e6, sizeof(unsigned short) * 3 * (size_t)NC * CD) != hipSuccess) {
        hipFree(tmp);
        return fail(h, DCX_ERR_OOM, "hipMalloc failed");
      }
      int rc = dcx::launch_split_planes(h->codebook, e6, NC, CD, 0, 0) == hipSuccess
                   ? DCX_OK : fail(h, DCX_ERR_HIP, "codebook split failed");
      const int mode = h->gemm_mode;
      h->gemm_mode = DCX_GEMM_BF16;
      ConvCall cp = pointwise(CAct(h->codebook, e6), NC);
      cp.y = tmp;
      if (rc == DCX_OK) rc = run_conv(h, pout, cp, 0);
      h->gemm_mode = mode;
      if (rc == DCX_OK &&
          (hipMemcpy(tmp + (size_t)NC * D, pout.b16, sizeof(float) * D, hipMemcpyDeviceToDevice) != hipSuccess ||
           dcx::launch_split_planes(tmp, h->ptable6b, NC + 1, D, 0, 0) != hipSuccess || hipDeviceSynchronize() != hipSuccess))
        rc = fail(h, DCX_ERR_HIP, "bf16 decode-table build failed");
      hipFree(e6);
      hipFree(tmp);
      if (rc != DCX_OK) return rc;
    }
    // the h3 range flags (round 6)
    if (!B.bad() && !B.dry) {
      h->rflag = (int*)B.alloc(1);
      if (!h->rflag || hipMemset(h->rflag, 0, sizeof(int)) != hipSuccess) return fail(h, DCX_ERR_HIP, "range flag");
    }
  }
  // ---- generator ------------------------------------------------------------------------
  if (with_generator) {
    const std::string g = "generator.";
    int ch = c.gen_channels;
    // h3 weights for the convs conv_gemm_x3dw takes (Cout % 256 == 0, or Cout % 128 == 0 on its
    // 384 x 128 tiles; two taps or more)
    h->conv_pre = B.conv(g + "conv_pre", c.vq_dim, ch, c.gen_pre_k, 1, (c.gen_pre_k - 1) / 2, true,
                         ch % 256 == 0 && c.gen_pre_k >= 2);
    for (int i = 0; i < c.n_ups; ++i) {
      h->ups[i] = B.convT(g + "ups." + std::to_string(i), ch, ch / 2, c.up_kernels[i], c.up_rates[i],
                          (ch / 2) % 128 == 0 && c.up_kernels[i] / c.up_rates[i] >= 2);
      ch /= 2;
      for (int rb = 0; rb < c.n_res; ++rb) {
        const int k = c.res_kernels[rb];
        for (int j = 0; j < 3; ++j) {
          const int d = c.res_dilations[rb][j];
          const std::string p = g + "resblocks." + std::to_string(i) + ".blocks." + std::to_string(rb);
          const bool h3 = ch % 32 == 0;  // conv_gemm_x3dq / x3dw tiles (C >= 128), conv_res_pair_h3 (32 / 64)
          h->res[i][rb][j][0] = B.conv(p + ".convs1." + std::to_string(j), ch, ch, k, d, (k * d - d) / 2, true, h3);
          h->res[i][rb][j][1] = B.conv(p + ".convs2." + std::to_string(j), ch, ch, k, 1, (k - 1) / 2, true, h3);
        }
      }
    }
    HostTensor pw = B.weight(g + "conv_post", {1, ch, c.gen_post_k});
    if (!B.bad()) {
      std::vector<float> pk((size_t)c.gen_post_k * ch);
      for (int i = 0; i < ch; ++i)
        for (int j = 0; j < c.gen_post_k; ++j) pk[(size_t)j * ch + i] = pw.data[(size_t)i * c.gen_post_k + j];
      h->post_w = B.upload(pk);
      auto pb = B.need(g + "conv_post.bias", {1});
      if (pb) h->post_b = pb->data[0];
    }
  }
  if (B.bad()) return fail(h, B.e.code, B.e.msg);
  return DCX_OK;
}

int dcx_finalize(dcx_codec* h, int32_t with_generator) {
  if (!h) return DCX_ERR_INVALID_ARG;
  if (h->finalized) return fail(h, DCX_ERR_STATE, "already finalized");
  Builder check{h, true};  // every required tensor present with the right size, before any upload
  int rc = build_all(h, check, with_generator);
  if (rc != DCX_OK) return rc;
  Builder B{h, false};
  rc = build_all(h, B, with_generator);
  if (rc != DCX_OK) return rc;
  h->has_gen = with_generator != 0;
  if (hipStreamCreateWithFlags(&h->side, hipStreamNonBlocking) != hipSuccess ||
      hipEventCreateWithFlags(&h->fork_ev, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&h->join_ev, hipEventDisableTiming) != hipSuccess)
    return fail(h, DCX_ERR_HIP, "dcx_finalize: stream / event creation failed");
  h->finalized = true;
  h->host.clear();
  return DCX_OK;
}

int64_t dcx_num_frames(const dcx_codec* h, int64_t n) { return h ? frames_of(h->cfg, n) : 0; }

size_t dcx_workspace_size(const dcx_codec* h, int32_t batch, int64_t frames) {
  if (!h || batch <= 0 || frames <= 0) return 0;
  dcx_codec* hh = const_cast<dcx_codec*>(h);
  const int64_t n = (frames - 1) * h->cfg.hop + h->cfg.n_fft - (h->cfg.win - h->cfg.hop);
  Bump d(nullptr, 0, true);
  stage_encode_decode(hh, nullptr, batch, n, nullptr, nullptr, d, 0);
  size_t need = d.off;
  Bump q(nullptr, 0, true);  // vq_encode with every optional output in the workspace
  stage_vq_encode(hh, CAct(), batch, (int)frames, nullptr, nullptr, nullptr, nullptr, q, 0);
  need = std::max(need, q.off + (size_t)batch * frames * (h->cfg.codebook_dim + h->cfg.vq_dim) * 4 + 1024);
  if (h->split_k > 1) need += kSplitScratch + 256;  // split-K partial sums (STAGE_PRE)
  return need + 4096;
}

// One stage call on a handle.  A handle is not re-entrant (the header's contract): a second call
// entering while one runs (another thread sharing the handle) is refused with DCX_ERR_STATE rather
// than left to overwrite the first call's split-K scratch pointer.  split_buf is cleared on exit, so
// no later call (or dcx_workspace_size's dry run) sees a pointer into another call's workspace.
struct CallScope {
  dcx_codec* h;
  bool owner = false;
  explicit CallScope(dcx_codec* hh) : h(hh) {
    int expect = 0;
    owner = h && h->busy.compare_exchange_strong(expect, 1);
  }
  ~CallScope() {
    if (owner) {
      h->split_buf = nullptr;
      h->busy.store(0);
    }
  }
};

#define STAGE_PRE(need_gen)                                           \
  int rc_ = check_ready(h, need_gen);                                 \
  if (rc_ != DCX_OK) return rc_;                                      \
  if (batch <= 0) return fail(h, DCX_ERR_INVALID_ARG, "batch must be > 0"); \
  CallScope scope_(h);                                                \
  if (!scope_.owner) return fail(h, DCX_ERR_STATE, "handle in use by a concurrent call (serialise calls per handle)"); \
  hipStream_t s = (hipStream_t)stream;                                \
  Bump ws(workspace, ws_bytes, false);                                \
  h->split_buf = h->split_k > 1 ? (float*)ws.raw(kSplitScratch) : nullptr

int dcx_mel(dcx_codec* h, const float* audio, int32_t batch, int64_t n, float* mel, void* workspace, size_t ws_bytes,
            void* stream) {
  STAGE_PRE(false);
  if (!audio || !mel) return fail(h, DCX_ERR_INVALID_ARG, "null buffer");
  if (n <= (h->cfg.win - h->cfg.hop) / 2 || frames_of(h->cfg, n) < 1)
    return fail(h, DCX_ERR_INVALID_ARG, "clip too short for the reflect pad / one STFT frame");
  return stage_mel(h, audio, batch, n, Act{mel, nullptr}, ws, s);
}

int dcx_mel_linear(dcx_codec* h, const float* audio, int32_t batch, int64_t n, float* mel, float* log_linear,
                   void* workspace, size_t ws_bytes, void* stream) {
  STAGE_PRE(false);
  if (!audio || !mel || !log_linear) return fail(h, DCX_ERR_INVALID_ARG, "null buffer");
  if (n <= (h->cfg.win - h->cfg.hop) / 2 || frames_of(h->cfg, n) < 1)
    return fail(h, DCX_ERR_INVALID_ARG, "clip too short for the reflect pad / one STFT frame");
  return stage_mel(h, audio, batch, n, Act{mel, nullptr}, ws, s, log_linear);
}

int dcx_encode(dcx_codec* h, const float* mel, int32_t batch, int64_t frames, float* feat, void* workspace,
               size_t ws_bytes, void* stream) {
  STAGE_PRE(false);
  if (!mel || !feat || frames <= 0) return fail(h, DCX_ERR_INVALID_ARG, "bad arguments");
  return stage_encode(h, CAct(mel, nullptr), batch, (int)frames, Act{feat, nullptr}, ws, s);
}

int dcx_vq_encode(dcx_codec* h, const float* feat, int32_t batch, int64_t frames, int32_t* codes, float* x_pjt_in,
                  float* quantized_fup, float* quantized, void* workspace, size_t ws_bytes, void* stream) {
  STAGE_PRE(false);
  if (!feat || !codes || frames <= 0) return fail(h, DCX_ERR_INVALID_ARG, "bad arguments");
  return stage_vq_encode(h, CAct(feat, nullptr), batch, (int)frames, codes, x_pjt_in, quantized_fup, quantized, ws, s);
}

int dcx_vq_decode(dcx_codec* h, const int32_t* codes, int32_t batch, int64_t frames, float* z, int32_t* n_invalid,
                  void* workspace, size_t ws_bytes, void* stream) {
  STAGE_PRE(false);
  if (!codes || !z || frames <= 0) return fail(h, DCX_ERR_INVALID_ARG, "bad arguments");
  return stage_vq_decode(h, codes, batch, (int)frames, Act{z, nullptr}, n_invalid, ws, s);
}

int dcx_generate(dcx_codec* h, const float* z, int32_t batch, int64_t frames, float* wav, void* workspace,
                 size_t ws_bytes, void* stream) {
  STAGE_PRE(true);
  if (!z || !wav || frames <= 0) return fail(h, DCX_ERR_INVALID_ARG, "bad arguments");
  return stage_generate(h, CAct(z, nullptr), batch, (int)frames, wav, ws, s);
}

int dcx_encode_decode(dcx_codec* h, const float* audio, int32_t batch, int64_t n, int32_t* codes, float* wav,
                      void* workspace, size_t ws_bytes, void* stream) {
  STAGE_PRE(true);
  if (!audio || !codes || !wav) return fail(h, DCX_ERR_INVALID_ARG, "null buffer");
  if (n <= (h->cfg.win - h->cfg.hop) / 2 || frames_of(h->cfg, n) < 1)
    return fail(h, DCX_ERR_INVALID_ARG, "clip too short for the reflect pad / one STFT frame");
  return stage_encode_decode(h, audio, batch, n, codes, wav, ws, s);
}

int dcx_module_io(const dcx_codec* h, const char* module, int32_t* in_channels, int32_t* out_channels,
                  int32_t* out_rate) {
  if (!h || !module) return DCX_ERR_INVALID_ARG;
  int ci = 0, co = 0, r = 1;
  // a read-only query: an unknown name returns DCX_ERR_INVALID_ARG without touching the handle's
  // last-error string (another thread may be running a stage call on the handle)
  if (!module_io(h, module, ci, co, r)) return DCX_ERR_INVALID_ARG;
  if (in_channels) *in_channels = ci;
  if (out_channels) *out_channels = co;
  if (out_rate) *out_rate = r;
  return DCX_OK;
}

size_t dcx_module_workspace_size(const dcx_codec* h, const char* module, int32_t batch, int64_t rows) {
  if (!h || !module || batch <= 0 || rows <= 0 || !h->finalized) return 0;
  Bump d(nullptr, 0, true);
  if (stage_module(const_cast<dcx_codec*>(h), module, nullptr, batch, (int)rows, nullptr, d, 0) != DCX_OK) return 0;
  // the split-K partial sums, carved ahead of the module's buffers (STAGE_PRE)
  return d.off + 4096 + (h->split_k > 1 ? kSplitScratch + 256 : 0);
}

int dcx_module_forward(dcx_codec* h, const char* module, const float* x, int32_t batch, int64_t rows,
                       int32_t channels, void* y, void* workspace, size_t ws_bytes, void* stream) {
  STAGE_PRE(false);
  if (!module || !x || !y || rows <= 0 || rows > (1 << 30)) return fail(h, DCX_ERR_INVALID_ARG, "bad arguments");
  int ci = 0, co = 0, r = 1;
  if (!module_io(h, module, ci, co, r)) return fail(h, DCX_ERR_INVALID_ARG, std::string("unknown module: ") + module);
  // the kernels read cin channels per row: any other width would be read out of bounds
  if (channels != ci)
    return fail(h, DCX_ERR_INVALID_ARG, std::string(module) + " takes " + std::to_string(ci) + " input channels, got " +
                                            std::to_string(channels));
  return stage_module(h, module, x, batch, (int)rows, y, ws, s);
}

int dcx_transpose(const float* in, float* out, int32_t batch, int64_t rows, int64_t cols, void* stream) {
  if (!in || !out || batch <= 0 || rows <= 0 || cols <= 0) return DCX_ERR_INVALID_ARG;
  return dcx::launch_transpose(in, out, batch, rows, cols, (hipStream_t)stream) == hipSuccess ? DCX_OK : DCX_ERR_HIP;
}

int dcx_resample_poly(const float* x, int32_t batch, int64_t n_in, int64_t x_stride, const double* h, int32_t h_len,
                      int32_t up, int32_t down, int64_t pre, float* y, int64_t n_out, int64_t y_stride, void* stream) {
  if (!x || !h || !y || batch <= 0 || n_in <= 0 || n_out <= 0 || h_len <= 0 || up <= 0 || down <= 0 || pre < 0 ||
      x_stride < n_in || y_stride < n_out || batch > 65535)
    return DCX_ERR_INVALID_ARG;
  // the largest filter index a thread can form must fit: t - up * m_lo < h_len by construction;
  // t itself must not overflow
  if ((pre + n_out) > (INT64_MAX / down)) return DCX_ERR_INVALID_ARG;
  return dcx::launch_resample_poly(x, batch, n_in, x_stride, h, h_len, up, down, pre, y, n_out, y_stride,
                                   (hipStream_t)stream) == hipSuccess
             ? DCX_OK
             : DCX_ERR_HIP;
}

int dcx_set_gemm_mode(dcx_codec* h, int32_t mode) {
  if (!h) return DCX_ERR_INVALID_ARG;
  if (mode != DCX_GEMM_F32 && mode != DCX_GEMM_X6 && mode != DCX_GEMM_BF16)
    return fail(h, DCX_ERR_INVALID_ARG, "unknown GEMM mode");
  h->gemm_mode = mode;
  return DCX_OK;
}

int32_t dcx_get_gemm_mode(const dcx_codec* h) { return h ? h->gemm_mode : -1; }

int dcx_set_split_k(dcx_codec* h, int32_t max_splits) {
  if (!h || max_splits < 0 || max_splits > kSplitMax) return DCX_ERR_INVALID_ARG;
  h->split_k = max_splits;
  return DCX_OK;
}

int dcx_set_knob(dcx_codec* h, const char* name, int32_t value) {
  if (!h || !name) return DCX_ERR_INVALID_ARG;
  // claim the handle as a stage call does (CallScope), so no call starts while the knob changes
  CallScope scope(h);
  if (!scope.owner) return fail(h, DCX_ERR_STATE, "dcx_set_knob during a stage call");
  int* k = knob_slot(h->knobs, name);
  if (!k) return fail(h, DCX_ERR_INVALID_ARG, std::string("unknown knob: ") + name);
  *k = value;
  return DCX_OK;
}

int dcx_get_knob(const dcx_codec* h, const char* name, int32_t* value) {
  if (!h || !name || !value) return DCX_ERR_INVALID_ARG;
  dcx::Knobs k = h->knobs;
  const int* slot = knob_slot(k, name);
  if (!slot) return DCX_ERR_INVALID_ARG;
  *value = *slot;
  return DCX_OK;
}

int dcx_range_flags(dcx_codec* h, int32_t* flags, int32_t reset) {
  if (!h || !flags) return DCX_ERR_INVALID_ARG;
  *flags = 0;
  if (!h->rflag) return DCX_OK;  // not finalized: no h3 call has run
  int v = 0;
  if (hipDeviceSynchronize() != hipSuccess || hipMemcpy(&v, h->rflag, sizeof v, hipMemcpyDeviceToHost) != hipSuccess)
    return fail(h, DCX_ERR_HIP, "reading the range flags failed");
  *flags = v;
  if (reset && hipMemset(h->rflag, 0, sizeof v) != hipSuccess) return fail(h, DCX_ERR_HIP, "resetting the range flags failed");
  return DCX_OK;
}

}  // extern "C"

struct dcx_conv {
  dcx_codec scratch;  // owns the device allocations and the last error
  ConvW w;
  unsigned short* planes = nullptr;  // x6 input planes of the last call (grown on demand)
  size_t planes_cap = 0;
};

extern "C" {

int dcx_conv_create(const float* weight, const float* bias, int32_t cin, int32_t cout, int32_t k, int32_t dilation,
                    int32_t transposed, int32_t stride, dcx_conv** out) {
  if (!weight || !out || cin <= 0 || cout <= 0 || k <= 0 || dilation <= 0 || stride <= 0) return DCX_ERR_INVALID_ARG;
  if (cin % 16 || cout % 32) return DCX_ERR_INVALID_ARG;
  if (transposed && (k % stride || (k - stride) % 2 || stride > dcx::kMaxPhases)) return DCX_ERR_INVALID_ARG;
  if (!transposed && (k % 2 == 0)) return DCX_ERR_INVALID_ARG;
  auto c = new (std::nothrow) dcx_conv();
  if (!c) return DCX_ERR_OOM;
  dcx_codec* h = &c->scratch;
  HostTensor wt;
  const int64_t n = (int64_t)cin * cout * k;
  wt.shape = transposed ? std::vector<int64_t>{cin, cout, k} : std::vector<int64_t>{cout, cin, k};
  wt.data.assign(weight, weight + n);
  h->host["c.weight"] = wt;
  HostTensor bt;
  bt.shape = {cout};
  if (bias) bt.data.assign(bias, bias + cout); else bt.data.assign(cout, 0.f);
  h->host["c.bias"] = bt;
  Builder B{h, false};
  c->w = transposed ? B.convT("c", cin, cout, k, stride) : B.conv("c", cin, cout, k, dilation, dilation * (k - 1) / 2);
  h->host.clear();
  if (B.bad()) {
    int code = B.e.code;
    dcx_conv_destroy(c);
    return code;
  }
  *out = c;
  return DCX_OK;
}

int dcx_conv_forward(dcx_conv* c, int32_t gemm_mode, const float* x, int32_t batch, int64_t lin, float* y,
                     float* y_silu, const float* res, int32_t epi, void* stream) {
  if (!c || !x || batch <= 0 || lin <= 0 || (!y && !y_silu)) return DCX_ERR_INVALID_ARG;
  if (epi != dcx::EPI_BIAS && epi != dcx::EPI_GELU && epi != dcx::EPI_RES) return DCX_ERR_INVALID_ARG;
  if (epi == dcx::EPI_RES && !res) return DCX_ERR_INVALID_ARG;
  dcx_codec* h = &c->scratch;
  h->gemm_mode = gemm_mode;
  hipStream_t s = (hipStream_t)stream;
  CAct xa(x, nullptr);
  if (gemm_mode != DCX_GEMM_F32 && gemm_mode != DCX_GEMM_X6 && gemm_mode != DCX_GEMM_BF16) return DCX_ERR_INVALID_ARG;
  if (gemm_mode != DCX_GEMM_F32 && !f32_input_ok(c->w)) {
    const size_t need = (size_t)batch * lin * c->w.cin * 3;
    if (need > c->planes_cap) {
      if (c->planes) hipFree(c->planes);
      c->planes = nullptr;
      c->planes_cap = 0;
      if (hipMalloc(&c->planes, need * sizeof(unsigned short)) != hipSuccess) return DCX_ERR_OOM;
      c->planes_cap = need;
    }
    if (dcx::launch_split_planes(x, c->planes, (long long)batch * lin, c->w.cin, 0, s) != hipSuccess) return DCX_ERR_HIP;
    xa.p = c->planes;
  }
  ConvCall cc = framed(xa, batch, (int)lin, c->w.cin);
  cc.y = y;
  cc.y2 = y_silu;
  cc.res = res;
  cc.epi = epi;
  return run_conv(h, c->w, cc, s);
}

void dcx_conv_destroy(dcx_conv* c) {
  if (!c) return;
  if (c->planes) hipFree(c->planes);
  for (void* p : c->scratch.allocs) hipFree(p);
  delete c;
}

int dcx_profile_enable(dcx_codec* h, int32_t on) {
  if (!h) return DCX_ERR_INVALID_ARG;
  h->prof = on != 0;
  return DCX_OK;
}

int dcx_profile_reset(dcx_codec* h) {
  if (!h) return DCX_ERR_INVALID_ARG;
  prof_collect(h);
  for (size_t i = 0; i < h->prof_names.size(); ++i) {
    h->prof_launches[i] = 0;
    h->prof_ms[i] = h->prof_flops[i] = h->prof_bytes[i] = 0;
  }
  return DCX_OK;
}

int dcx_vq_rescore_stats(dcx_codec* h, int64_t* rows_rescored, int64_t* codes_rescored, int32_t reset) {
  if (!h || !h->vq_stats) return DCX_ERR_STATE;
  h->vq_stats_on = true;
  int v[2] = {0, 0};
  if (hipDeviceSynchronize() != hipSuccess || hipMemcpy(v, h->vq_stats, sizeof v, hipMemcpyDeviceToHost) != hipSuccess)
    return fail(h, DCX_ERR_HIP, "reading VQ rescore counters failed");
  if (rows_rescored) *rows_rescored = v[0];
  if (codes_rescored) *codes_rescored = v[1];
  if (reset && hipMemset(h->vq_stats, 0, sizeof v) != hipSuccess)
    return fail(h, DCX_ERR_HIP, "resetting VQ rescore counters failed");
  return DCX_OK;
}

int32_t dcx_profile_count(const dcx_codec* h) { return h ? (int32_t)h->prof_names.size() : 0; }

int dcx_profile_read(dcx_codec* h, int32_t i, const char** name, int64_t* launches, double* ms, double* flops,
                     double* bytes) {
  if (!h) return DCX_ERR_INVALID_ARG;
  prof_collect(h);
  if (i < 0 || i >= (int32_t)h->prof_names.size()) return DCX_ERR_INVALID_ARG;
  if (name) *name = h->prof_names[i].c_str();
  if (launches) *launches = h->prof_launches[i];
  if (ms) *ms = h->prof_ms[i];
  if (flops) *flops = h->prof_flops[i];
  if (bytes) *bytes = h->prof_bytes[i];
  return DCX_OK;
}

}  // extern "C"
