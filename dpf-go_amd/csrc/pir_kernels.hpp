// pir_kernels.hpp — launcher for the PIR answer fold (pir_kernels.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace dpfk {

// ans[k][0..7] ^= XOR of the 32-byte records db[i] (i < nrec) whose bit i is
// set in bits[k * words_per_key ...].  `parts` is scratch of
// pir_fold_parts_bytes() (per-wave partial answers).
uint64_t pir_fold_parts_bytes();
hipError_t launch_pir_fold(const uint32_t* bits, uint64_t words_per_key, const uint8_t* db, uint64_t nrec,
                           uint32_t nkeys, uint32_t* ans, uint32_t* parts, hipStream_t st);

}  // namespace dpfk
