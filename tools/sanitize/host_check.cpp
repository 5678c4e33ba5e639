// Host-only sanitizer driver for the runtime's native host code (ops/csrc/host.hip): built by
// tools/sanitize/run_host_asan.sh with AddressSanitizer + UBSan on the host side only and run on the CPU
// (SURVEY.md §5.2).  Exercises dtf_crc32c over every length/alignment of a heap buffer allocated to its exact
// size, so an over-read of one byte past the end is reported by ASan, and checks the RFC 3720 test vectors.
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

extern "C" uint32_t dtf_crc32c(const uint8_t* p, size_t n, uint32_t crc);

static uint32_t crc32c_ref(const uint8_t* p, size_t n, uint32_t crc) {
  uint32_t c = ~crc;
  for (size_t i = 0; i < n; ++i) {
    c ^= p[i];
    for (int k = 0; k < 8; ++k) c = (c >> 1) ^ (0x82F63B78u & (0u - (c & 1u)));
  }
  return ~c;
}

int main(int argc, char** argv) {
  if (argc > 1 && std::strcmp(argv[1], "--canary") == 0) {
    // self-test of the instrumentation: a one-byte heap over-read that ASan must report (non-zero exit)
    uint8_t* buf = static_cast<uint8_t*>(std::malloc(13));
    std::memset(buf, 1, 13);
    uint32_t c = dtf_crc32c(buf, 14, 0);
    std::free(buf);
    std::printf("canary not caught (%08x)\n", c);
    return 0;
  }
  int fails = 0;
  // RFC 3720 B.4 vectors
  std::vector<uint8_t> z(32, 0), o(32, 0xff), inc(32), dec(32);
  for (int i = 0; i < 32; ++i) inc[i] = (uint8_t)i, dec[i] = (uint8_t)(31 - i);
  const struct { const std::vector<uint8_t>* v; uint32_t want; } vecs[] = {
      {&z, 0x8A9136AAu}, {&o, 0x62A8AB43u}, {&inc, 0x46DD794Eu}, {&dec, 0x113FDB5Cu}};
  for (auto& t : vecs) {
    uint32_t got = dtf_crc32c(t.v->data(), t.v->size(), 0);
    if (got != t.want) { std::printf("vector mismatch: %08x != %08x\n", got, t.want); ++fails; }
  }
  // every length 0..300 at every start offset 0..7, in an exact-size heap block (ASan redzone right after it)
  for (size_t n = 0; n <= 300; ++n) {
    for (size_t off = 0; off < 8; ++off) {
      uint8_t* buf = static_cast<uint8_t*>(std::malloc(off + n + 1)) ;
      for (size_t i = 0; i < off + n; ++i) buf[i] = (uint8_t)(i * 131 + n);
      uint32_t seed = (uint32_t)(n * 2654435761u);
      uint32_t a = dtf_crc32c(buf + off, n, seed), b = crc32c_ref(buf + off, n, seed);
      if (a != b) { if (fails < 10) std::printf("n=%zu off=%zu: %08x != %08x\n", n, off, a, b); ++fails; }
      std::free(buf);
    }
  }
  std::printf("host_check: %s (%d failures)\n", fails ? "FAIL" : "ok", fails);
  return fails ? 1 : 0;
}
