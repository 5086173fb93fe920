// pir_kernels.hpp — launcher for the XOR fold (pir_kernels.hip): the PIR
// answer and the general-payload streaming consumer of EvalFull output.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define DPF_FOLD_PLAN 1   // plan_fold() below (tools/fold_bench.hip)

namespace dpfk {

// How launch_pir_fold covers (rec_bytes, nkeys): `cols` 32-byte columns per
// pass (1, 2, 4 or 8 = the whole record; 1 with `col_passes` = rec_bytes/32
// for other widths), `keys_per_pass` keys per DB read, the direct kernel or
// Four-Russians with `kw` 64-key lane groups sharing each table.
struct FoldPlan {
    uint32_t cols, col_passes, keys_per_pass, kw;
    bool direct;
};
FoldPlan plan_fold(uint64_t rec_bytes, uint32_t nkeys);

// ans[k][0 .. rec_bytes) = XOR of the records db[i] (rec_bytes each, a
// multiple of 32; i < nrec) whose bit i is set in bits[k * words_per_key
// ...] (EvalFull's LSB-first layout); zero when nrec == 0.  The first fold
// launch clears ans itself (no separate memset).  `parts` is scratch of
// pir_fold_parts_bytes() (per-workgroup partial answers).  bits, db 16-byte
// aligned; words_per_key a multiple of 4 covering nrec bits.
uint64_t pir_fold_parts_bytes();
hipError_t launch_pir_fold(const uint32_t* bits, uint64_t words_per_key, const uint8_t* db, uint64_t nrec,
                           uint64_t rec_bytes, uint32_t nkeys, uint32_t* ans, uint32_t* parts, hipStream_t st);

// The MFMA fold (k_fold_mfma, 32-byte records): the same answers from the DB
// in its bit-sliced layout (dbs, pir_sliced_bytes(nrec) bytes, built once by
// launch_slice_db from the row-major DB).  Same bits / parts / ans contract
// as launch_pir_fold.
uint64_t pir_sliced_bytes(uint64_t nrec);
hipError_t launch_slice_db(const uint8_t* db, uint64_t nrec, uint8_t* dbs, hipStream_t st);
// sgm_keys > 0: the selection bits are super-group-major instead, in chunks
// of sgm_g (1 or 4) super-groups: bits[S / g][sgm_keys][g * 8 words]
// (S < ceil(nrec / 256)); key k of the batch is row k.
hipError_t launch_pir_fold_sliced(const uint32_t* bits, uint64_t words_per_key, const uint8_t* dbs, uint64_t nrec,
                                  uint32_t nkeys, uint32_t* ans, uint32_t* parts, hipStream_t st,
                                  uint32_t sgm_keys = 0, uint32_t sgm_g = 1);

// Tuning / test limits of the fold launches: at most max_blocks workgroups
// per launch (0 = the default, 1024), and at most max_sg super-groups per
// matrix-core fold workgroup (0 = the default and maximum, 2^15 = 2^23
// records, so its fp32 counts stay below 2^24); larger DBs fold in passes.
void set_fold_limits(uint32_t max_blocks, uint32_t max_sg);

// Fused PIR answer (k_pir_fused): the subtree EvalFull of keys [0, nkeys)
// from their expanded records (launch_unpack) and the matrix-core fold over
// the sliced DB in one launch; where pir_fused_ok() (<= 64 keys, 2^8 .. 2^10
// blocks of 256 leaf pairs in the subtree; any_size: from one block, for
// tests).  Same ans / parts contract.  Built only with DPF_PIR_FUSED_KERNEL=1
// (make experimental): measured slower than the two launches;
// otherwise pir_fused_ok() is false and the launcher refuses.
bool pir_fused_ok(uint64_t nkeys, uint32_t stop, uint32_t prefix_bits, bool any_size = false);
// Whether k_pir_fused is compiled into this library (the experimental build only).
bool pir_fused_built();
hipError_t launch_pir_fused(const uint32_t* ek, uint32_t nkeys, uint32_t stop, uint32_t prefix_bits, uint64_t prefix,
                            const uint8_t* dbs, uint64_t nrec, uint32_t* ans, uint32_t* parts, hipStream_t st);

}  // namespace dpfk
