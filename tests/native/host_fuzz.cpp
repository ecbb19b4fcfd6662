// Host-side fuzz of the C ABI entry points that run without a GPU, built with
// AddressSanitizer + UndefinedBehaviorSanitizer on the host code (Makefile target `asan`):
//   * ef_jpeg_info — the JPEG marker parser (DQT/DHT/SOF/DRI/SOS, restart segments) that
//     every batched decode runs on untrusted files: each seed file plus deterministic
//     mutations (bit flips, 0xFF / marker-byte injection, length-field tampering,
//     truncation, splices), one file per call and all of them in one batch call;
//   * ef_matches_merge (host form) and ef_keys_decode on random records.
// A sanitizer report aborts the process (non-zero exit); tests/test_host_sanitizers.py
// runs it on Pillow-encoded seeds.  usage: host_fuzz <iterations> <seed.jpg>...
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <iterator>
#include <random>
#include <vector>

#include "../../include/eigenface.h"

static std::vector<uint8_t> read_file(const char* p) {
  std::ifstream f(p, std::ios::binary);
  return std::vector<uint8_t>((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
}

static std::vector<uint8_t> mutate(const std::vector<uint8_t>& s, std::mt19937_64& rng) {
  std::vector<uint8_t> m = s;
  if (m.empty()) return m;
  const int kind = (int)(rng() % 7);
  const size_t n = m.size();
  switch (kind) {
    case 0:  // bit flips anywhere
      for (int i = 0, k = 1 + (int)(rng() % 8); i < k; ++i) m[rng() % n] ^= (uint8_t)(1u << (rng() % 8));
      break;
    case 1:  // 0xFF injection (fake markers / stuffing)
      for (int i = 0, k = 1 + (int)(rng() % 4); i < k; ++i) m[rng() % n] = 0xFF;
      break;
    case 2: {  // tamper a marker's length field
      std::vector<size_t> at;
      for (size_t i = 0; i + 3 < n; ++i)
        if (m[i] == 0xFF && m[i + 1] >= 0xC0 && m[i + 1] != 0xFF && m[i + 1] != 0xD8) at.push_back(i);
      if (!at.empty()) {
        const size_t i = at[rng() % at.size()];
        const uint16_t v = (uint16_t)rng();
        m[i + 2] = (uint8_t)(v >> 8);
        m[i + 3] = (uint8_t)v;
      }
      break;
    }
    case 3:  // truncation
      m.resize(rng() % n);
      break;
    case 4: {  // splice a random chunk of itself elsewhere
      const size_t a = rng() % n, b = rng() % n, len = 1 + rng() % 64;
      for (size_t i = 0; i < len && a + i < n && b + i < n; ++i) m[b + i] = m[a + i];
      break;
    }
    case 5: {  // marker byte swap (SOF -> SOF2, DHT class/id, DQT precision)
      for (size_t i = 0; i + 1 < n; ++i)
        if (m[i] == 0xFF && (m[i + 1] == 0xC0 || m[i + 1] == 0xC4 || m[i + 1] == 0xDB || m[i + 1] == 0xDA) &&
            rng() % 3 == 0) {
          if (i + 4 < n) m[i + 4] = (uint8_t)rng();
        }
      break;
    }
    default:  // random byte values in the header region
      for (int i = 0, k = 1 + (int)(rng() % 16); i < k; ++i) m[rng() % std::min<size_t>(n, 700)] = (uint8_t)rng();
      break;
  }
  return m;
}

int main(int argc, char** argv) {
  if (argc < 3) {
    std::fprintf(stderr, "usage: %s <iterations> <seed.jpg>...\n", argv[0]);
    return 2;
  }
  const int iters = std::atoi(argv[1]);
  std::vector<std::vector<uint8_t>> seeds;
  for (int i = 2; i < argc; ++i) seeds.push_back(read_file(argv[i]));
  std::mt19937_64 rng(12345);
  long ok = 0, rejected = 0;
  std::vector<std::vector<uint8_t>> batch;
  for (int it = 0; it < iters; ++it) {
    const auto& s = seeds[it % seeds.size()];
    std::vector<uint8_t> m = it < (int)seeds.size() ? s : mutate(s, rng);
    if (it % 5 == 0 && !m.empty()) m = mutate(m, rng);  // stacked mutations
    // one file per call (exact-size heap buffer, so reads past it are caught)
    std::vector<uint8_t> own(m.begin(), m.end());
    const int64_t off = 0, sz = (int64_t)own.size();
    int32_t h = 0, w = 0, c = 0, st = 0;
    const int rc = ef_jpeg_info(own.empty() ? nullptr : own.data(), &off, &sz, own.empty() ? 0 : 1, &h, &w, &c, &st);
    if (rc != EF_OK) return 3;
    (st == 0 ? ok : rejected)++;
    if (batch.size() < 512) batch.push_back(std::move(m));
  }
  // the batch form (shared table dedup across files)
  std::vector<uint8_t> all;
  std::vector<int64_t> offs, sizes;
  for (auto& b : batch) {
    offs.push_back((int64_t)all.size());
    sizes.push_back((int64_t)b.size());
    all.insert(all.end(), b.begin(), b.end());
  }
  std::vector<int32_t> H(batch.size()), W(batch.size()), Cc(batch.size()), S(batch.size());
  if (!batch.empty() && !all.empty())
    if (ef_jpeg_info(all.data(), offs.data(), sizes.data(), (int32_t)batch.size(), H.data(), W.data(), Cc.data(),
                     S.data()) != EF_OK)
      return 4;
  // host merge of random match records, and key decoding
  for (int t = 0; t < 200; ++t) {
    const int nparts = 1 + (int)(rng() % 8);
    const int64_t b = 1 + (int64_t)(rng() % 300);
    std::vector<ef_match> parts((size_t)nparts * b);
    std::uniform_real_distribution<double> u(-10.0, 10.0);
    for (auto& r : parts) {
      r.score = (rng() % 17 == 0) ? __builtin_inf() : u(rng);
      r.scale = std::fabs(u(rng));
      r.key = (rng() % 17 == 0) ? INT64_MAX : (int64_t)(rng() & 0x7fffffffffffffffULL);
    }
    std::vector<int64_t> keys(b);
    std::vector<ef_match> merged(b);
    if (ef_matches_merge(nullptr, parts.data(), nparts, b, keys.data(), merged.data(), 0) != EF_OK) return 5;
    std::vector<float> best(b);
    std::vector<int64_t> idx(b);
    ef_keys_decode(keys.data(), b, (int32_t)(t & 1), best.data(), idx.data());
  }
  std::printf("host_fuzz: %d files (%ld parsed, %ld rejected), batch of %zu, 200 merges: clean\n", iters, ok, rejected,
              batch.size());
  return 0;
}
