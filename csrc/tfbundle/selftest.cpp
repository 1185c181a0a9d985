// Host-side self-test of the TF-bundle codec, built with -fsanitize=address,undefined by
// tests/test_sanitizers_cpu.py (the C++ codec runs under ASan/UBSan in the test suite).
//
//   selftest <prefix-of-a-reference-bundle> <scratch-dir>
//
// Checks (exit 0 = all passed, 1 = a check failed; ASan/UBSan abort on a memory error or undefined behaviour):
//   1. CRC32C test vectors (RFC 3720), incremental CRCs at every split point, mask/unmask round trips;
//   2. the reference demo checkpoint: parse -> rebuild the index byte-identically; read -> write -> both files
//      byte-identical;
//   3. corruption: a flipped data byte raises a checksum FormatError; every single-byte flip of the index parses or
//      raises FormatError (never another exception);
//   4. every truncation of the index raises FormatError;
//   5. a deterministic fuzz of parse_index (random bytes, varint continuation bytes, deletions);
//   6. block handles and tensor extents near 2^64 / 2^63 (the overflow cases of off + size) raise FormatError.
#include <cstdint>
#include <cstdio>
#include <fstream>
#include <sstream>
#include <string>
#include <vector>

#include "tf_bundle.h"

namespace {

int g_fail = 0;

#define CHECK(cond, ...)                                          \
  do {                                                            \
    if (!(cond)) {                                                \
      std::fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__);   \
      std::fprintf(stderr, __VA_ARGS__);                          \
      std::fprintf(stderr, "\n");                                 \
      ++g_fail;                                                   \
    }                                                             \
  } while (0)

std::string slurp(const std::string& p) {
  std::ifstream f(p, std::ios::binary);
  std::ostringstream ss;
  ss << f.rdbuf();
  return ss.str();
}

void spit(const std::string& p, const std::string& s) {
  std::ofstream f(p, std::ios::binary | std::ios::trunc);
  f.write(s.data(), (std::streamsize)s.size());
}

// 0 = parsed, 1 = FormatError, 2 = any other exception
int try_parse(const std::string& bytes) {
  try {
    tfb::Header h;
    std::vector<tfb::Entry> e;
    tfb::parse_index(bytes, &h, &e);
    return 0;
  } catch (const tfb::FormatError&) {
    return 1;
  } catch (...) {
    return 2;
  }
}

uint64_t g_lcg = 0x9E3779B97F4A7C15ull;
uint32_t rnd() {
  g_lcg = g_lcg * 6364136223846793005ull + 1442695040888963407ull;
  return (uint32_t)(g_lcg >> 33);
}

void put_varint(std::string* s, uint64_t v) {
  while (v >= 0x80) {
    s->push_back((char)((v & 0x7F) | 0x80));
    v >>= 7;
  }
  s->push_back((char)v);
}

void test_crc() {
  const char* nine = "123456789";
  CHECK(tfb::crc32c((const uint8_t*)nine, 9) == 0xE3069283u, "crc32c(123456789)");
  std::vector<uint8_t> z(32, 0), f(32, 0xFF), inc(32), dec(32);
  for (int i = 0; i < 32; ++i) {
    inc[i] = (uint8_t)i;
    dec[i] = (uint8_t)(31 - i);
  }
  CHECK(tfb::crc32c(z.data(), 32) == 0x8A9136AAu, "crc32c(32 x 00)");
  CHECK(tfb::crc32c(f.data(), 32) == 0x62A8AB43u, "crc32c(32 x ff)");
  CHECK(tfb::crc32c(inc.data(), 32) == 0x46DD794Eu, "crc32c(0..31)");
  CHECK(tfb::crc32c(dec.data(), 32) == 0x113FDB5Cu, "crc32c(31..0)");
  for (int s = 0; s <= 32; ++s) {   // slicing-by-8 head / tail paths
    const uint32_t a = tfb::crc32c(inc.data() + s, 32 - s, tfb::crc32c(inc.data(), s));
    CHECK(a == 0x46DD794Eu, "incremental crc split at %d", s);
  }
  for (int i = 0; i < 1000; ++i) {
    const uint32_t c = rnd() ^ (rnd() << 16);
    CHECK(tfb::unmask_crc(tfb::mask_crc(c)) == c, "mask round trip");
  }
}

void test_demo(const std::string& prefix, const std::string& scratch) {
  const std::string idx = slurp(prefix + ".index");
  const std::string dat = slurp(prefix + ".data-00000-of-00001");
  CHECK(!idx.empty() && !dat.empty(), "demo bundle missing at %s", prefix.c_str());
  if (idx.empty() || dat.empty()) return;
  tfb::Header h;
  std::vector<tfb::Entry> entries;
  tfb::parse_index(idx, &h, &entries);
  CHECK(!entries.empty(), "demo has entries");
  CHECK(tfb::build_index(h, entries) == idx, "rebuilt index is byte-identical");
  std::vector<tfb::Tensor> ts = tfb::read_bundle(prefix, true);
  CHECK(ts.size() == entries.size(), "read_bundle entry count");
  const std::string out = scratch + "/selftest_rewrite";
  tfb::write_bundle(out, ts);
  CHECK(slurp(out + ".index") == idx, "rewritten index is byte-identical");
  CHECK(slurp(out + ".data-00000-of-00001") == dat, "rewritten data is byte-identical");

  std::string bad = dat;
  bad[bad.size() / 2] ^= 0x20;
  const std::string cp = scratch + "/selftest_corrupt";
  spit(cp + ".index", idx);
  spit(cp + ".data-00000-of-00001", bad);
  bool raised = false;
  try {
    tfb::read_bundle(cp, true);
  } catch (const tfb::FormatError&) {
    raised = true;
  }
  CHECK(raised, "a corrupted data byte raises FormatError");
  bool ok = true;
  try {
    tfb::read_bundle(cp, false);
  } catch (...) {
    ok = false;
  }
  CHECK(ok, "verify_crc=false reads a corrupted payload");

  for (size_t i = 0; i < idx.size(); ++i) {
    std::string m = idx;
    m[i] ^= 0x5A;
    CHECK(try_parse(m) != 2, "byte flip at %zu raised a non-FormatError exception", i);
  }
  for (size_t n = 0; n < idx.size(); ++n) CHECK(try_parse(idx.substr(0, n)) == 1, "truncation to %zu parsed", n);
  for (int it = 0; it < 20000; ++it) {
    std::string m = idx;
    const int k = 1 + (int)(rnd() % 8);
    for (int j = 0; j < k && !m.empty(); ++j) {
      const size_t at = rnd() % m.size();
      switch (rnd() % 4) {
        case 0: m[at] = (char)rnd(); break;
        case 1: m[at] = (char)0xFF; break;           // varint continuation bytes
        case 2: m[at] = (char)0x80; break;
        default: m.erase(at, 1 + rnd() % 4); break;  // deletions shift every later field
      }
    }
    CHECK(try_parse(m) != 2, "mutation %d raised a non-FormatError exception", it);
  }
}

// footer pointing at a block handle whose off + size + trailer overflows 64 bits
void test_handle_overflow() {
  const uint64_t sizes[] = {~0ull, ~0ull - 4, ~0ull - 5, 1ull << 63, (1ull << 63) - 1, 0xFFFFFFFFull};
  const uint64_t offs[] = {0ull, 1ull, 7ull, ~0ull};
  for (uint64_t off : offs) {
    for (uint64_t sz : sizes) {
      std::string f(64, '\0');
      std::string footer;
      put_varint(&footer, 0);
      put_varint(&footer, 0);
      put_varint(&footer, off);
      put_varint(&footer, sz);
      footer.resize(40, '\0');
      const uint64_t magic = 0xdb4775248b80fb57ull;
      for (int i = 0; i < 8; ++i) footer.push_back((char)((magic >> (8 * i)) & 0xFF));
      f += footer;
      CHECK(try_parse(f) == 1, "block handle (%llu, %llu) accepted", (unsigned long long)off, (unsigned long long)sz);
    }
  }
}

// an entry whose extent offset + size overflows int64
void test_extent_overflow(const std::string& scratch) {
  const int64_t offs[] = {0, 1, (int64_t)(1ull << 62), INT64_MAX, INT64_MAX - 3};
  const int64_t sizes[] = {4, (int64_t)(1ull << 62), INT64_MAX, INT64_MAX - 1};
  for (int64_t off : offs) {
    for (int64_t sz : sizes) {
      tfb::Entry e;
      e.key = "x";
      e.dtype = 1;
      e.shape = {1};
      e.offset = off;
      e.size = sz;
      e.crc32c = 0;
      tfb::Header h;
      const std::string p = scratch + "/selftest_extent";
      spit(p + ".index", tfb::build_index(h, {e}));
      spit(p + ".data-00000-of-00001", std::string(8, '\0'));
      int outcome = 0;
      try {
        tfb::read_bundle(p, true);
      } catch (const tfb::FormatError&) {
        outcome = 1;
      } catch (...) {
        outcome = 2;
      }
      const bool fits = off >= 0 && sz >= 0 && off <= 8 && sz <= 8 - off;
      CHECK(fits ? outcome != 2 : outcome == 1, "extent (%lld, %lld) -> outcome %d", (long long)off, (long long)sz,
            outcome);
    }
  }
}

}  // namespace

int main(int argc, char** argv) {
  if (argc < 3) {
    std::fprintf(stderr, "usage: %s <reference-bundle-prefix> <scratch-dir>\n", argv[0]);
    return 2;
  }
  test_crc();
  test_demo(argv[1], argv[2]);
  test_handle_overflow();
  test_extent_overflow(argv[2]);
  if (g_fail) {
    std::fprintf(stderr, "%d check(s) failed\n", g_fail);
    return 1;
  }
  std::printf("tfbundle selftest: all checks passed\n");
  return 0;
}
