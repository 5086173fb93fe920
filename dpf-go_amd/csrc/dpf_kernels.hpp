// dpf_kernels.hpp — launchers for the gfx950 DPF kernels (dpf_kernels.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace dpfk {

constexpr int kBlock = 512;    // threads per workgroup (8 waves); 2 workgroups per CU (64 KiB LDS table each)
#ifndef DPF_TREE_BLOCK
#define DPF_TREE_BLOCK 512
#endif
#ifndef DPF_TREE_WAVES
#define DPF_TREE_WAVES 4
#endif
#ifndef DPF_TREE_BLOCK_BIG
#define DPF_TREE_BLOCK_BIG 1024
#endif
// Tree kernel geometry: 2 workgroups of kTreeBlock threads per CU (LDS-bound),
// kTreeWaves waves per SIMD (VGPR budget).  Leaf launches with deep
// per-thread subtrees (D >= kBigMinD: configs[1], configs[3]) use one
// kTreeBlockBig-thread workgroup per CU instead, so that all 16 waves of a CU
// share one LDS and can balance their progress (prio_step feedback form).
// Build-time knobs for A/B runs.
constexpr int kTreeBlock = DPF_TREE_BLOCK;
constexpr int kTreeBlockBig = DPF_TREE_BLOCK_BIG;
constexpr int kTreeBlockMax = kTreeBlock > kTreeBlockBig ? kTreeBlock : kTreeBlockBig;
#ifndef DPF_BIG_MIN_D
#define DPF_BIG_MIN_D 6
#endif
constexpr uint32_t kBigMinD = DPF_BIG_MIN_D;
#ifndef DPF_FEEDBACK_MIN_D
#define DPF_FEEDBACK_MIN_D 6
#endif
constexpr uint32_t kFeedbackMinD = DPF_FEEDBACK_MIN_D;   // progress feedback needs enough groups per thread
constexpr int kTreeWaves = DPF_TREE_WAVES;
constexpr uint32_t kMaxD = 7;  // per-thread DFS subtree depth: 128 leaves = 2 KiB of output per thread
constexpr uint32_t kMaxFrontierHbm = 16;  // batched Eval, HBM frontier: deepest shared level

// CU budget of the calling thread's launches (0: the whole device); see
// cu_count() in dpf_kernels.hip.
void set_cu_budget(int cus);
int cu_budget();
int cu_count();

// Expanded-key words per key: (stop + 2) records of 8 u32.
inline uint64_t ek_words(uint32_t stop) { return ((uint64_t)stop + 2) * 8; }

// aes128MMO iterated `reps` times over nblocks (even) blocks, T-table back end.
hipError_t launch_mmo_tt(const uint8_t* in, uint8_t* out, uint64_t nblocks, uint32_t right, uint32_t reps,
                         hipStream_t st);

hipError_t launch_unpack(const uint8_t* keys, uint64_t key_len, uint64_t nkeys, uint32_t stop, uint32_t* ek,
                         hipStream_t st);

// EvalFull of the subtree rooted at depth `prefix_bits`, index `prefix`, of
// every key (prefix_bits = 0 -> whole domain).  Output per key: 2^(stop -
// prefix_bits) leaves of 16 B at out + key * out_stride.
hipError_t launch_evalfull(const uint32_t* ek, uint64_t nkeys, uint32_t stop, uint32_t prefix_bits,
                           uint64_t prefix, uint8_t* out, uint64_t out_stride, hipStream_t st);

// The same from the key bytes themselves ([nkeys][klen], the reference's
// layout, any alignment), no unpack launch: only where evalfull_raw_ok()
// (every wave owns one key).
bool evalfull_raw_ok(uint64_t nkeys, uint32_t stop, uint32_t prefix_bits);
hipError_t launch_evalfull_raw(const uint8_t* keys, uint64_t klen, uint64_t nkeys, uint32_t stop, uint32_t prefix_bits,
                               uint64_t prefix, uint8_t* out, uint64_t out_stride, hipStream_t st);

// The 2^(depth - prefix_bits) nodes at level `depth` below prefix node
// (prefix_bits, prefix) of every key: seeds (16 B) at seeds + (key * stride
// + j) * 16 and t bytes at ts + key * stride + j.
hipError_t launch_nodes(const uint32_t* ek, uint64_t nkeys, uint32_t stop, uint32_t depth, uint32_t prefix_bits,
                        uint64_t prefix, uint8_t* seeds, uint8_t* ts, uint64_t stride, hipStream_t st);

// Batched Eval.  When a key has enough points to share the top of its tree
// (L = the deepest level with 2^(L+1) <= pts_per_key, used when L >= 4), the
// 2^L nodes at level L of every key are first
// computed into `frontier` (eval_frontier_bytes of it) and each query starts
// there; with frontier == nullptr (or too small) every walk starts at the root.
uint32_t eval_frontier_level(uint32_t stop, uint64_t pts_per_key);
// Batched Eval kernel choice: 1 = visited-node trie below the frontier.
int set_eval_trie(int on);   // returns the previous choice
int get_eval_trie();
bool eval_trie_built();   // k_eval_trie is in this build (the experimental one)
uint64_t eval_frontier_bytes(uint64_t nkeys, uint32_t stop, uint64_t pts_per_key);
hipError_t launch_eval(const uint32_t* ek, uint32_t stop, uint32_t logN, const uint64_t* xs, uint64_t nq,
                       uint64_t pts_per_key, uint8_t* out, void* frontier, uint64_t frontier_bytes,
                       hipStream_t st);

}  // namespace dpfk
