// Host-side memory-safety run of the C ABI (built with ASan + UBSan by `make asan`; no GPU
// needed): the RIFF/WAVE walk (mgx_wav_parse) over a seeded fuzz corpus of valid files of
// every format and mutations of them (truncation at every length, byte flips, chunk sizes
// 0 / odd / huge, fmt chunks of 14-40 bytes, chunks in any order, no data), each handed over
// in a heap block of exactly its length so any over-read is caught; the host tables for
// every power-of-two buffer size up to 65536 and every mel-band / coefficient count, into
// exactly-sized buffers; shard and packed-layout arithmetic; descriptor and argument
// validation (the reference validates its inputs at src/meyda.js:20-26).
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

#include "../../include/meyda_gpu.h"

static int failures = 0;
#define CHECK(c)                                                         \
  do {                                                                   \
    if (!(c)) {                                                          \
      fprintf(stderr, "%s:%d: check failed: %s\n", __FILE__, __LINE__, #c); \
      ++failures;                                                        \
    }                                                                    \
  } while (0)

static void put16(std::vector<uint8_t>& b, uint16_t v) { b.push_back(v & 255); b.push_back(v >> 8); }
static void put32(std::vector<uint8_t>& b, uint32_t v) { for (int i = 0; i < 4; ++i) b.push_back((v >> (8 * i)) & 255); }
static void tag(std::vector<uint8_t>& b, const char* t) { b.insert(b.end(), t, t + 4); }

// A WAVE file: fmt chunk of fmt_size bytes (16, 18 or 40), optional extra chunk, data.
static std::vector<uint8_t> wav(uint16_t fmt_tag, uint16_t ch, uint16_t bits, uint32_t frames, uint32_t fmt_size,
                                bool extra_first, std::mt19937& rng) {
  std::vector<uint8_t> b;
  tag(b, "RIFF");
  put32(b, 0);
  tag(b, "WAVE");
  auto extra = [&]() {
    tag(b, "LIST");
    const uint32_t n = rng() % 7;
    put32(b, n);
    for (uint32_t i = 0; i < n; ++i) b.push_back(rng() & 255);
    if (n & 1) b.push_back(0);
  };
  if (extra_first) extra();
  tag(b, "fmt ");
  put32(b, fmt_size);
  const uint16_t align = ch * (bits / 8);
  put16(b, fmt_size == 40 ? 0xFFFE : fmt_tag);
  put16(b, ch);
  put32(b, 44100);
  put32(b, 44100u * align);
  put16(b, align);
  put16(b, bits);
  if (fmt_size >= 18) put16(b, fmt_size - 18);
  if (fmt_size == 40) {
    put16(b, bits);
    put32(b, 3);
    put16(b, fmt_tag);
    for (int i = 0; i < 14; ++i) b.push_back(0);
  }
  if (!extra_first) extra();
  tag(b, "data");
  put32(b, frames * align);
  for (uint32_t i = 0; i < frames * align; ++i) b.push_back(rng() & 255);
  const uint32_t riff = (uint32_t)b.size() - 8;
  memcpy(&b[4], &riff, 4);
  return b;
}

static void parse_exact(const std::vector<uint8_t>& bytes, size_t len) {
  uint8_t* p = static_cast<uint8_t*>(malloc(len ? len : 1));
  if (len) memcpy(p, bytes.data(), len);
  mgx_wav_info wi;
  memset(&wi, 0, sizeof wi);
  wi.struct_size = sizeof wi;
  if (mgx_wav_parse(p, len, &wi) == MGX_OK) {
    CHECK(wi.data_offset + wi.data_bytes <= len);
    CHECK(wi.block_align > 0 && wi.data_bytes % wi.block_align == 0);
    CHECK(wi.sample_frames * wi.block_align == wi.data_bytes);
    CHECK(wi.channels > 0);
  }
  free(p);
}

static void wav_fuzz() {
  std::mt19937 rng(0x6D657964);
  const struct { uint16_t t, bits; } fmts[] = {{1, 8}, {1, 16}, {1, 24}, {1, 32}, {3, 32}};
  long n = 0;
  for (const auto& f : fmts)
    for (uint16_t ch : {1, 2, 5})
      for (uint32_t fs : {16u, 18u, 40u})
        for (bool ex : {false, true}) {
          const std::vector<uint8_t> good = wav(f.t, ch, f.bits, 1 + rng() % 9, fs, ex, rng);
          mgx_wav_info wi;
          memset(&wi, 0, sizeof wi);
          wi.struct_size = sizeof wi;
          CHECK(mgx_wav_parse(good.data(), good.size(), &wi) == MGX_OK);
          for (size_t len = 0; len <= good.size(); ++len, ++n) parse_exact(good, len);  // every truncation
          for (int m = 0; m < 200; ++m, ++n) {                                       // random mutations
            std::vector<uint8_t> b = good;
            const int kind = rng() % 4;
            const size_t at = rng() % b.size();
            if (kind == 0) b[at] ^= (uint8_t)(1u << (rng() % 8));
            else if (kind == 1 && b.size() >= 4) {  // a chunk size field: 0, odd, huge, all ones
              const uint32_t vals[] = {0u, 1u, 0x7FFFFFFFu, 0xFFFFFFFFu, (uint32_t)b.size(), 13u};
              const uint32_t v = vals[rng() % 6];
              const size_t pos = std::min(at, b.size() - 4);
              memcpy(&b[pos], &v, 4);
            } else if (kind == 2) {
              b.resize(at);
            } else {
              b.insert(b.begin() + at, (size_t)(rng() % 5), (uint8_t)(rng() & 255));
            }
            parse_exact(b, b.size());
          }
        }
  // a fmt chunk shorter than 16 bytes, a data chunk first, no chunks at all
  std::vector<uint8_t> b;
  tag(b, "RIFF"); put32(b, 20); tag(b, "WAVE"); tag(b, "fmt "); put32(b, 14);
  for (int i = 0; i < 14; ++i) b.push_back(1);
  parse_exact(b, b.size());
  b.clear();
  tag(b, "RIFF"); put32(b, 12); tag(b, "WAVE"); tag(b, "data"); put32(b, 4); put32(b, 0);
  parse_exact(b, b.size());
  b.resize(12);
  parse_exact(b, b.size());
  printf("wav_parse: %ld buffers\n", n);
}

static void host_tables() {
  long n = 0;
  for (uint32_t N = 1; N <= 65536; N <<= 1)
    for (uint32_t nf : {1u, 2u, 26u, 40u, 64u})
      for (uint32_t nc : {1u, 13u, 32u}) {
        mgx_plan_desc d;
        mgx_plan_desc_init(&d);
        d.buffer_size = N;
        d.num_mel_bands = nf;
        d.num_mfcc_coeffs = nc;
        std::vector<float> win(N), han(N), ham(N), bark(N), dct((size_t)nf * nc);
        std::vector<int32_t> lim(25), bins(nf + 2);
        mgx_host_tables t = {win.data(), han.data(), ham.data(), bark.data(), lim.data(), bins.data(), dct.data()};
        CHECK(mgx_get_host_tables(&d, &t) == MGX_OK);
        CHECK(lim[24] == (int32_t)(N / 2) - 1);
        ++n;
      }
  mgx_plan_desc d;
  mgx_plan_desc_init(&d);
  d.buffer_size = 1000;
  mgx_host_tables t = {};
  CHECK(mgx_get_host_tables(&d, &t) == MGX_E_NOT_POWER_OF_TWO);
  CHECK(mgx_get_host_tables(nullptr, &t) == MGX_E_INVALID_ARGUMENT);
  printf("host tables: %ld plans\n", n);
}

static void arithmetic() {
  for (uint64_t total : {0ull, 1ull, 7ull, 262144ull, 2097155ull})
    for (uint32_t R : {1u, 3u, 8u}) {
      uint64_t next = 0;
      for (uint32_t r = 0; r < R; ++r) {
        uint64_t s, c;
        CHECK(mgx_shard_range(total, R, r, &s, &c) == MGX_OK);
        CHECK(s == next);
        next = s + c;
      }
      CHECK(next == total);
    }
  uint64_t s, c;
  CHECK(mgx_shard_range(5, 0, 0, &s, &c) != MGX_OK);
  CHECK(mgx_shard_range(5, 2, 2, &s, &c) != MGX_OK);
  mgx_plan_desc d;
  mgx_plan_desc_init(&d);
  uint64_t off[19];
  CHECK(mgx_packed_layout(&d, MGX_OUT_ALL_MASK, 1000, off) > 0);
  for (int i = 1; i < 19; ++i) CHECK(off[i] > off[i - 1] && off[i] % 256 == 0);
  CHECK(mgx_packed_layout(nullptr, 1, 1, off) == 0);
  CHECK(mgx_feature_index(nullptr) == -1);
  CHECK(mgx_feature_index("") == -1);
  CHECK(mgx_feature_name(-1) == nullptr && mgx_feature_name(19) == nullptr);
  CHECK(mgx_is_power_of_two(0.0) == 0 && mgx_is_power_of_two(1.0) == 1 && mgx_is_power_of_two(-8.0) == 0);
}

static void validation() {
  mgx_plan* p = nullptr;
  CHECK(mgx_plan_create(nullptr, &p) == MGX_E_INVALID_ARGUMENT);
  mgx_plan_desc d;
  mgx_plan_desc_init(&d);
  d.struct_size = 4;
  CHECK(mgx_plan_create(&d, &p) == MGX_E_INVALID_ARGUMENT);
  mgx_plan_desc_init(&d);
  d.flags = 0x80;
  CHECK(mgx_plan_create(&d, &p) == MGX_E_INVALID_ARGUMENT);
  mgx_plan_desc_init(&d);
  d.num_mel_bands = 65;
  CHECK(mgx_plan_create(&d, &p) == MGX_E_UNSUPPORTED);
  mgx_group* g = nullptr;
  CHECK(mgx_group_create(&d, nullptr, 0, &g) == MGX_E_INVALID_ARGUMENT);
  CHECK(mgx_group_create_rank(&d, nullptr, 2, 5, &g) == MGX_E_INVALID_ARGUMENT);
  CHECK(mgx_extract_host_pcm(nullptr, nullptr, 0, 0, 0, 0, 0, nullptr) == MGX_E_INVALID_ARGUMENT);
  CHECK(strlen(mgx_last_error()) > 0);
}

int main() {
  wav_fuzz();
  host_tables();
  arithmetic();
  validation();
  printf("host_checks: %s (%d failures)\n", failures ? "FAILED" : "ok", failures);
  return failures ? 1 : 0;
}
