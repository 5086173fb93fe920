// pir_kernels.hpp — launcher for the PIR answer fold (pir_kernels.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace dpfk {

// ans[k][0 .. rec_bytes) ^= XOR of the records db[i] (rec_bytes each, a
// multiple of 32; i < nrec) whose bit i is set in bits[k * words_per_key
// ...] (EvalFull's LSB-first layout).  `parts` is scratch of
// pir_fold_parts_bytes() (per-workgroup partial answers).
uint64_t pir_fold_parts_bytes();
hipError_t launch_pir_fold(const uint32_t* bits, uint64_t words_per_key, const uint8_t* db, uint64_t nrec,
                           uint64_t rec_bytes, uint32_t nkeys, uint32_t* ans, uint32_t* parts, hipStream_t st);

}  // namespace dpfk
