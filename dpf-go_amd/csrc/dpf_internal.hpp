// dpf_internal.hpp — shared declarations inside libdpf_hip.so.
#pragma once
#include <stddef.h>
#include <stdint.h>

namespace dpfh {

inline uint32_t stop_of(uint32_t logN) { return logN >= 7 ? logN - 7 : 0; }
inline size_t key_len(uint32_t logN) { return 33 + 18 * (size_t)stop_of(logN); }
inline size_t full_len(uint32_t logN) { return logN > 63 ? 0 : logN >= 7 ? ((size_t)1 << (logN - 3)) : 16; }   // 0: no such output
// Bit `s` of x with Go's shift semantics: Eval's path test
// `x & (uint64(1) << (logN-1-i))` (dpf.go:194) is 0 once the shift reaches
// 64, so a logN > 63 key takes the left child on its top logN-64 levels.
inline uint32_t path_bit(uint64_t x, uint64_t s) { return s < 64 ? (uint32_t)((x >> s) & 1u) : 0u; }

bool host_has_aesni();
int gen_seeded(uint64_t alpha, uint32_t logN, const uint8_t s0[16], const uint8_t s1[16], uint8_t* ka, uint8_t* kb);
int gen_random(uint64_t alpha, uint32_t logN, uint8_t* ka, uint8_t* kb);
int gen_batch_seeded(const uint64_t* alphas, uint32_t logN, const uint8_t* s0s, const uint8_t* s1s, size_t n,
                     uint8_t* kas, uint8_t* kbs, int nthreads);
int keys_pack(const uint8_t* const* keys, const size_t* lens, size_t n, size_t key_len, uint8_t* out);
int keys_unpack(const uint8_t* packed, size_t key_len, size_t n, uint8_t* const* keys);

// host_eval.cpp: the single-call path (AES-NI / VAES), bit-exact with the kernels.
bool host_eval_available();
bool host_eval_vaes();   // the EvalFull host path runs on VAES (else 128-bit AES-NI)
void eval_batch_host(const uint8_t* keys, size_t klen, size_t nkeys, const uint64_t* xs, size_t ppk, uint32_t logN,
                     uint8_t* out);
void evalfull_host(const uint8_t* key, size_t klen, uint32_t logN, uint8_t* out);

}  // namespace dpfh
