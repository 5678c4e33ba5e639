// Host-side helpers of the runtime (no device code): CRC32C (Castagnoli) for the TensorFlow tensor-bundle
// checkpoint writer (utils/tf_bundle.py) -- SSE4.2 crc32 instructions, 8 bytes per step.
#include <cstddef>
#include <cstdint>
#include <cstring>
#include <nmmintrin.h>

extern "C" __attribute__((visibility("default"), target("sse4.2"))) uint32_t dtf_crc32c(const uint8_t* p, size_t n,
                                                                                        uint32_t crc) {
  uint64_t c = ~crc;
  while (n >= 8) {
    uint64_t v;
    std::memcpy(&v, p, 8);
    c = _mm_crc32_u64(c, v);
    p += 8;
    n -= 8;
  }
  uint32_t c32 = (uint32_t)c;
  while (n--) c32 = _mm_crc32_u8(c32, *p++);
  return ~c32;
}

// Build configuration of the loaded library, so the Python side sizes its buffers from what was actually compiled
// (not from environment variables that may disagree with it): BatchNorm-statistic replicas per member and BN
// (common.h DTF_NREP) and whether this is the deterministic build (fixed-order reductions).
#ifndef DTF_NREP
#define DTF_NREP 8
#endif
extern "C" __attribute__((visibility("default"))) int dtf_nrep() { return DTF_NREP; }
extern "C" __attribute__((visibility("default"))) int dtf_build_deterministic() {
#ifdef DTF_DETERMINISTIC
  return 1;
#else
  return 0;
#endif
}
// 1: the half build (-DDTF_HALF: fp16 activation / weight-shadow storage, v_mfma_f32_16x16x32_f16), selected by
// --dtype fp16 (DTF_HALF=1); 0: bf16
extern "C" __attribute__((visibility("default"))) int dtf_build_half() {
#ifdef DTF_HALF
  return 1;
#else
  return 0;
#endif
}
