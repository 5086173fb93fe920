// bs_kernels.hpp — EvalFull with the byte-sliced AES back end (bs_kernels.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace dpfk {

// Levels a lane expands below the frontier (2^D leaves per node): 4, or 3
// when 4 would leave CUs idle (bs_depth).
constexpr uint32_t kBsDMax = 4;
constexpr uint32_t kBsDMin = 3;

// Block order inside a set of 8 consecutive nodes: after an expansion at
// depth d (shift s_d = 4, 2, 1 cycling, P_d = {p : (p & s_d) == 0}), block p
// in P_d holds child 2*sigma(p) and block p + s_d child 2*sigma(p) + 1.
struct Sigma {
    uint32_t v[8];
};
constexpr Sigma sigma_at(uint32_t depth) {
    Sigma s = {{0, 1, 2, 3, 4, 5, 6, 7}};
    for (uint32_t d = 0; d < depth; ++d) {
        const uint32_t sh = d % 3 == 0 ? 4 : d % 3 == 1 ? 2 : 1;
        Sigma n = {};
        for (uint32_t p = 0; p < 8; ++p)
            if ((p & sh) == 0) {                 // invariant: s.v[p] < 4 here (nodes 0..3 sit in P_d)
                n.v[p] = s.v[p] < 4 ? 2 * s.v[p] : 99;
                n.v[p + sh] = n.v[p] + 1;
            }
        s = n;
    }
    return s;
}
constexpr bool sigma_ok(uint32_t depth) {
    for (uint32_t d = 0; d <= depth; ++d)
        for (uint32_t p = 0; p < 8; ++p)
            if (sigma_at(d).v[p] >= 8) return false;
    return true;
}
static_assert(sigma_ok(12), "set block order invariant");
static_assert(sigma_at(4).v[0] == 0 && sigma_at(4).v[1] == 2 && sigma_at(4).v[4] == 1, "sigma(4) = [0,2,4,6,1,3,5,7]");
static_assert(sigma_at(3).v[5] == 5, "sigma(3) = identity");

__host__ __device__ uint64_t bs_key_words(uint32_t stop);   // byte-sliced correction words per key
bool bs_applicable(uint32_t stop, uint32_t prefix_bits);
uint32_t bs_depth(uint64_t nkeys, uint32_t stop, uint32_t prefix_bits);
uint64_t bs_frontier_bytes(uint64_t nkeys, uint32_t stop, uint32_t prefix_bits);

// T-table records (ek, k_unpack's layout) and byte-sliced records (ekb) in one launch.
// Byte-sliced records from the T-table records (ek) already in a workspace.
hipError_t launch_bs_from_ek(const uint32_t* ek, uint64_t nkeys, uint32_t stop, uint32_t* ekb, hipStream_t st);
hipError_t launch_unpack_both(const uint8_t* keys, uint64_t key_len, uint64_t nkeys, uint32_t stop, uint32_t* ek,
                              uint32_t* ekb, hipStream_t st);
hipError_t launch_unpack_bs(const uint8_t* keys, uint64_t key_len, uint64_t nkeys, uint32_t stop, uint32_t* ekb,
                            hipStream_t st);
// EvalFull of subtree (prefix_bits, prefix) of every key through the
// byte-sliced back end: ek = T-table key records (frontier pass), ekb =
// byte-sliced words (launch_unpack_bs), frontier = bs_frontier_bytes scratch.
hipError_t launch_evalfull_bs(const uint32_t* ek, const uint32_t* ekb, uint64_t nkeys, uint32_t stop,
                              uint32_t prefix_bits, uint64_t prefix, uint8_t* out, uint64_t out_stride, void* frontier,
                              hipStream_t st);
hipError_t launch_mmo_bs(const uint8_t* in, uint8_t* out, uint64_t nblocks, uint32_t key, uint32_t reps,
                         hipStream_t st);

}  // namespace dpfk
