// Host-code sanitizer driver (AddressSanitizer + UndefinedBehaviorSanitizer) for libdcx's host
// runtime: the C ABI's argument checks, checkpoint ingestion (name / shape validation, weight-norm
// folding, packing), workspace planning over many shapes and modes, and the MP3 decoder on its
// demo input, every prefix of it and thousands of corrupted copies.  Built by `make -C
// distilcodec_nabeel_amd/csrc sanitize` (dcx_api.cpp and dcx_mp3.cpp instrumented on the host,
// the kernels linked as built); run by tests/test_sanitize.py.  Without a GPU, dcx_finalize fails
// at its first device allocation (after the dry validation pass) and the stage calls are only
// checked for their argument errors; with one, a small encode_decode runs too.
//
//   host_driver mp3 FILE.mp3
//   host_driver abi TENSORS.txt      (lines: name ndim d0 d1 ...; the reference's state-dict keys)
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <sstream>
#include <string>
#include <vector>

#include <hip/hip_runtime.h>

#include "../../include/distilcodec_amd.h"

static int g_fail = 0;
#define CHECK(cond)                                                    \
  do {                                                                 \
    if (!(cond)) {                                                     \
      std::fprintf(stderr, "CHECK failed at line %d: %s\n", __LINE__, #cond); \
      ++g_fail;                                                        \
    }                                                                  \
  } while (0)

static uint64_t g_rng = 0x9E3779B97F4A7C15ull;
static uint32_t rnd() {
  g_rng ^= g_rng << 13;
  g_rng ^= g_rng >> 7;
  g_rng ^= g_rng << 17;
  return (uint32_t)(g_rng >> 11);
}

static std::vector<uint8_t> read_file(const char* path) {
  std::ifstream f(path, std::ios::binary);
  return std::vector<uint8_t>((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
}

static int decode_any(const std::vector<uint8_t>& d) {
  int64_t n = 0;
  int32_t sr = 0, ch = 0;
  const int rc = dcx_mp3_info(d.data(), d.size(), &n, &sr, &ch);
  if (rc != DCX_OK) return rc;
  if (n < 0 || n > (int64_t)1 << 28) return -100;
  std::vector<float> out((size_t)std::max<int64_t>(n * std::max(ch, 1), 1));
  return dcx_mp3_decode(d.data(), d.size(), out.data(), (int64_t)out.size());
}

static int run_mp3(const char* path) {
  const std::vector<uint8_t> d = read_file(path);
  CHECK(!d.empty());
  CHECK(decode_any(d) == DCX_OK);
  int64_t gr = 0, ex = 0;
  CHECK(dcx_mp3_stats(&gr, &ex) == DCX_OK && gr > 0 && gr == ex);
  // prefixes (every 509 bytes, then the last 64 one by one)
  for (size_t n = 0; n < d.size(); n += (n + 64 < d.size() ? 509 : 1))
    decode_any(std::vector<uint8_t>(d.begin(), d.begin() + n));
  // corrupted copies: 1-16 random byte / bit flips anywhere
  for (int it = 0; it < 400; ++it) {
    std::vector<uint8_t> c = d;
    const int k = 1 + rnd() % 16;
    for (int j = 0; j < k; ++j) {
      const size_t pos = rnd() % c.size();
      if (rnd() & 1) c[pos] ^= (uint8_t)(1u << (rnd() % 8));
      else c[pos] = (uint8_t)rnd();
    }
    decode_any(c);
  }
  // junk runs inserted anywhere (the scan resyncs on confirmed headers; damaged frames are silenced)
  for (int it = 0; it < 100; ++it) {
    std::vector<uint8_t> c = d;
    std::vector<uint8_t> junk(1 + rnd() % 2000);
    for (auto& b : junk) b = (uint8_t)rnd();
    c.insert(c.begin() + rnd() % c.size(), junk.begin(), junk.end());
    decode_any(c);
  }
  // garbage and frame-sync lookalikes
  for (int it = 0; it < 200; ++it) {
    std::vector<uint8_t> g(1 + rnd() % 4096);
    for (auto& b : g) b = (uint8_t)rnd();
    for (size_t p = 0; p + 1 < g.size(); p += 1 + rnd() % 400) { g[p] = 0xFF; g[p + 1] = 0xFB; }
    decode_any(g);
  }
  CHECK(dcx_mp3_info(nullptr, 10, nullptr, nullptr, nullptr) != DCX_OK);
  float tiny[4];
  CHECK(dcx_mp3_decode(d.data(), d.size(), tiny, 4) != DCX_OK);  // capacity below the sample count
  std::printf("mp3: %zu bytes, 110 prefixes, 400 corrupted, 100 junk-inserted and 200 garbage inputs decoded or rejected\n", d.size());
  return g_fail;
}

struct Spec {
  std::string name;
  std::vector<int64_t> shape;
};

static std::vector<Spec> read_specs(const char* path) {
  std::vector<Spec> out;
  std::ifstream f(path);
  std::string line;
  while (std::getline(f, line)) {
    std::istringstream is(line);
    Spec s;
    int nd = 0;
    if (!(is >> s.name >> nd)) continue;
    s.shape.resize(nd);
    for (int i = 0; i < nd; ++i) is >> s.shape[i];
    out.push_back(s);
  }
  return out;
}

static int set_all(dcx_codec* h, const std::vector<Spec>& specs, int skip, int bad_shape) {
  int rc = DCX_OK;
  for (int i = 0; i < (int)specs.size(); ++i) {
    if (i == skip) continue;
    const Spec& s = specs[i];
    int64_t n = 1;
    for (auto v : s.shape) n *= v;
    std::vector<float> data((size_t)std::max<int64_t>(n, 1));
    const float scale = 1.0f / std::sqrt((float)std::max<int64_t>(s.shape.empty() ? 1 : s.shape.back(), 1));
    for (auto& x : data) x = ((int)(rnd() % 2001) - 1000) * 1e-3f * scale;
    std::vector<int64_t> shape = s.shape;
    if (i == bad_shape && !shape.empty()) shape[0] += 1, data.resize(data.size() + data.size() / std::max<int64_t>(s.shape[0], 1) + 1);
    const int r = dcx_set_tensor(h, s.name.c_str(), data.data(), (int32_t)shape.size(), shape.data());
    if (r != DCX_OK) rc = r;
  }
  return rc;
}

static int run_abi(const char* specs_path) {
  const std::vector<Spec> specs = read_specs(specs_path);
  CHECK(specs.size() > 100);
  dcx_config c;
  dcx_default_config(&c);
  // invalid configurations are refused before anything is allocated
  for (int m = 0; m < 6; ++m) {
    dcx_config b = c;
    if (m == 0) b.n_fft = 512;
    if (m == 1) b.enc_dims[2] = 300;
    if (m == 2) b.up_rates[0] = 3;
    if (m == 3) b.n_ups = 9;
    if (m == 4) b.codebook_size = 100;
    if (m == 5) b.res_kernels[1] = 4;
    dcx_codec* hb = nullptr;
    CHECK(dcx_create(&b, &hb) == DCX_ERR_INVALID_ARG && hb == nullptr);
  }
  CHECK(dcx_create(nullptr, nullptr) == DCX_ERR_INVALID_ARG);

  dcx_codec* h = nullptr;
  CHECK(dcx_create(&c, &h) == DCX_OK && h);
  int64_t shp[2] = {2, -1};
  float v[4] = {0, 0, 0, 0};
  CHECK(dcx_set_tensor(h, nullptr, v, 1, shp) != DCX_OK);
  CHECK(dcx_set_tensor(h, "encoder.x", v, 2, shp) != DCX_OK);  // negative extent
  CHECK(dcx_set_tensor(h, "encoder.x", nullptr, 1, shp) != DCX_OK);
  CHECK(set_all(h, specs, -1, -1) == DCX_OK);
  // stage calls before finalize: state errors, nothing touched
  int32_t codes[4];
  float buf[64];
  CHECK(dcx_encode_decode(h, buf, 1, 48000, codes, buf, buf, 64, nullptr) == DCX_ERR_STATE);
  const int fin = dcx_finalize(h, 1);
  int ndev = 0;
  const bool gpu = hipGetDeviceCount(&ndev) == hipSuccess && ndev > 0;
  std::printf("finalize: %d (%s)\n", fin, gpu ? "GPU present" : "no GPU: the first device allocation fails");
  CHECK(gpu ? fin == DCX_OK : fin != DCX_OK);
  CHECK(dcx_finalize(nullptr, 1) == DCX_ERR_INVALID_ARG);

  // workspace planning over shapes, modes and the split-K setting (dry passes, no device work)
  size_t last = 0;
  for (int mode : {DCX_GEMM_X6, DCX_GEMM_BF16, DCX_GEMM_F32})
    for (int sk : {0, 16}) {
      CHECK(dcx_set_gemm_mode(h, mode) == DCX_OK);
      CHECK(dcx_set_split_k(h, sk) == DCX_OK);
      for (int B : {1, 2, 3, 32, 256})
        for (int64_t T : {1, 2, 3, 93, 139, 937, 2000}) {
          const size_t w = dcx_workspace_size(h, B, T);
          CHECK(w > 0);
          last ^= w;
        }
    }
  CHECK(dcx_set_gemm_mode(h, 7) != DCX_OK);
  CHECK(dcx_set_split_k(h, 17) != DCX_OK && dcx_set_split_k(h, -1) != DCX_OK);
  CHECK(dcx_set_split_k(h, 0) == DCX_OK && dcx_set_gemm_mode(h, DCX_GEMM_X6) == DCX_OK);
  CHECK(dcx_workspace_size(h, 0, 10) == 0 && dcx_workspace_size(nullptr, 1, 10) == 0);
  for (int64_t n : {0, 1, 383, 384, 385, 640, 24001, 240001}) last ^= (size_t)dcx_num_frames(h, n);

  if (gpu && fin == DCX_OK) {  // one small encode_decode through the instrumented host runtime
    const int B = 2;
    const int64_t n = 24001;
    const int64_t T = dcx_num_frames(h, n);
    const size_t wsz = dcx_workspace_size(h, B, T);
    float *audio = nullptr, *wav = nullptr;
    int32_t* dcodes = nullptr;
    void* ws = nullptr;
    CHECK(hipMalloc(&audio, B * n * 4) == hipSuccess && hipMalloc(&wav, B * T * 256 * 4) == hipSuccess &&
          hipMalloc(&dcodes, B * T * 4) == hipSuccess && hipMalloc(&ws, wsz) == hipSuccess);
    std::vector<float> ha(B * n);
    for (auto& x : ha) x = ((int)(rnd() % 2001) - 1000) * 2e-4f;
    CHECK(hipMemcpy(audio, ha.data(), ha.size() * 4, hipMemcpyHostToDevice) == hipSuccess);
    CHECK(dcx_encode_decode(h, audio, B, n, dcodes, wav, ws, 1 << 20, nullptr) == DCX_ERR_WORKSPACE);
    CHECK(dcx_encode_decode(h, audio, B, n, dcodes, wav, ws, wsz, nullptr) == DCX_OK);
    CHECK(dcx_encode_decode(h, audio, B, 100, dcodes, wav, ws, wsz, nullptr) == DCX_ERR_INVALID_ARG);
    std::vector<int32_t> hc(B * T);
    CHECK(hipMemcpy(hc.data(), dcodes, hc.size() * 4, hipMemcpyDeviceToHost) == hipSuccess);
    for (auto x : hc) CHECK(x >= 0 && x < c.codebook_size);
    (void)hipFree(audio);
    (void)hipFree(wav);
    (void)hipFree(dcodes);
    (void)hipFree(ws);
  }
  dcx_destroy(h);

  // a missing tensor and a mis-shaped tensor are reported by the dry validation pass
  dcx_codec* h2 = nullptr;
  CHECK(dcx_create(&c, &h2) == DCX_OK);
  set_all(h2, specs, (int)(rnd() % specs.size()), -1);
  CHECK(dcx_finalize(h2, 1) == DCX_ERR_MISSING_WEIGHT);
  dcx_destroy(h2);
  dcx_codec* h3 = nullptr;
  CHECK(dcx_create(&c, &h3) == DCX_OK);
  set_all(h3, specs, -1, 0);
  const int r3 = dcx_finalize(h3, 1);
  CHECK(r3 == DCX_ERR_INVALID_ARG || r3 == DCX_ERR_MISSING_WEIGHT);
  dcx_destroy(h3);

  // the standalone conv primitive: argument checks, then creation (device allocation)
  std::vector<float> w(64 * 32 * 3);
  for (auto& x : w) x = ((int)(rnd() % 201) - 100) * 1e-3f;
  dcx_conv* cv = nullptr;
  CHECK(dcx_conv_create(w.data(), nullptr, 32, 64, 4, 1, 0, 1, &cv) == DCX_ERR_INVALID_ARG);  // even k
  CHECK(dcx_conv_create(w.data(), nullptr, 30, 64, 3, 1, 0, 1, &cv) == DCX_ERR_INVALID_ARG);  // cin % 16
  const int rc = dcx_conv_create(w.data(), nullptr, 32, 64, 3, 1, 0, 1, &cv);
  CHECK(gpu ? rc == DCX_OK : rc != DCX_OK);
  if (cv) dcx_conv_destroy(cv);
  double taps[8] = {0};
  CHECK(dcx_resample_poly(nullptr, 1, 10, 10, taps, 8, 1, 2, 0, nullptr, 5, 5, nullptr) != DCX_OK);
  std::printf("abi: %zu tensors, plans checked (%zx)\n", specs.size(), last);
  return g_fail;
}

int main(int argc, char** argv) {
  if (argc == 3 && std::strcmp(argv[1], "mp3") == 0) return run_mp3(argv[2]) ? 1 : 0;
  if (argc == 3 && std::strcmp(argv[1], "abi") == 0) return run_abi(argv[2]) ? 1 : 0;
  std::fprintf(stderr, "usage: host_driver mp3 FILE | abi TENSORS.txt\n");
  return 2;
}
