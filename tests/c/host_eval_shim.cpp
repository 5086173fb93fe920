// host_eval_shim.cpp — C entry points over the library's host small-call
// path (dpf-go_amd/csrc/host_eval.cpp), linked by tests/test_capi.py into a
// throwaway .so so the CPU suite can check it against the oracle without a
// GPU (the product entry points dpf_eval / dpf_evalfull require an open
// gfx950 device before they route to it).
#include <stddef.h>
#include <stdint.h>

#include "../../dpf-go_amd/csrc/dpf_internal.hpp"

extern "C" {
int shim_available(void) { return dpfh::host_eval_available() ? 1 : 0; }
void shim_evalfull(const uint8_t* key, size_t klen, uint32_t logN, uint8_t* out) {
    dpfh::evalfull_host(key, klen, logN, out);
}
void shim_eval_batch(const uint8_t* keys, size_t klen, size_t nkeys, const uint64_t* xs, size_t ppk, uint32_t logN,
                     uint8_t* out) {
    dpfh::eval_batch_host(keys, klen, nkeys, xs, ppk, logN, out);
}
}
