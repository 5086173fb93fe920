/*
 * dpf_hip.h — C ABI of the MI355X DPF evaluation engine (libdpf_hip.so).
 *
 * Drop-in boundary for dkales/dpf-go's evaluation path.  The reference's Go
 * API is (dpf/dpf.go):
 *     type DPFkey []byte                                  :7
 *     func Gen(alpha, logN uint64) (DPFkey, DPFkey)       :71
 *     func Eval(k DPFkey, x, logN uint64) byte            :171
 *     func EvalFull(key DPFkey, logN uint64) []byte       :243
 * A cgo file in package dpf keeps those signatures and calls the functions
 * below.  Byte layouts are the reference's, unchanged:
 *   key   = seed[16] | t[1] | stop x (sCW[16] | tLCW[1] | tRCW[1]) | finalCW[16]
 *           stop = max(logN-7, 0), length 33 + 18*stop      (dpf.go:89-167)
 *   EvalFull output = 2^(logN-3) bytes (16 if logN < 7), point x is bit
 *           (x % 8) of byte (x / 8)                          (dpf.go:248-251, dpf_test.go:52)
 *
 * Conventions: every buffer is caller-owned; calls are synchronous unless
 * the name ends in _dev; nothing is retained after return (cgo pointer
 * rules).  Return value 0 = success, negative = error (DPF_ERR_*); the Go
 * wrapper turns a nonzero code into panic(), as the reference panics.
 * All functions are thread-safe (per-device mutex + stream).
 */
#ifndef DPF_HIP_H
#define DPF_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define DPF_OK 0
#define DPF_ERR_PARAM (-1)   /* invalid alpha/logN: where Gen panics (dpf.go:72-74) */
#define DPF_ERR_KEYLEN (-2)  /* key shorter than 17+18*stop: where Eval/EvalFull index out of range */
#define DPF_ERR_NODEV (-3)   /* no usable gfx950 device / dpf_gpu_init not possible */
#define DPF_ERR_HIP (-4)     /* HIP runtime error (message in dpf_last_error) */
#define DPF_ERR_NOMEM (-5)   /* device or host allocation failed */

/* Last error message of the calling thread ("" if none). */
const char* dpf_last_error(void);

/* ---- sizes ------------------------------------------------------------ */
/* len(DPFkey) produced by Gen for this logN (dpf.go:89-167). */
size_t dpf_key_len(uint32_t logN);
/* len(EvalFull(k, logN)) (dpf.go:248-251); 0 for logN > 63 (no such output). */
size_t dpf_evalfull_len(uint32_t logN);
/* Device scratch bytes the _dev entry points need for nkeys keys. */
size_t dpf_workspace_size(size_t nkeys, uint32_t logN);

/* ---- device management (no reference counterpart: the reference has no
 *      device; dpf.go:22-44 init() is the nearest analogue) --------------- */
/* Open ngpus devices (<= 0: every visible device).  Idempotent.  Returns the
 * number of devices opened (> 0) or a negative error.  Host-buffer entry
 * points open every visible device on first use when nothing is open. */
int dpf_gpu_init(int ngpus);
/* Open exactly the HIP ordinals ordinals[0..n) (e.g. one process per GPU:
 * its LOCAL_RANK only), so no context is created on any other device.
 * Idempotent for the same list; DPF_ERR_PARAM if other devices are open. */
int dpf_gpu_init_devices(const int* ordinals, int n);
/* Drops the library's references to the opened devices.  Calls already in
 * flight and live PIR handles keep the devices they use until they finish
 * (or are freed); later host-buffer calls re-open devices on demand. */
void dpf_gpu_shutdown(void);
int dpf_gpu_count(void);

/* ---- host-side key generation (Gen stays on the host, north star) ------ */
/* Replaces Gen (dpf.go:71-169) with the two crypto/rand seeds (:80-81)
 * passed in.  ka/kb: dpf_key_len(logN) bytes each. */
int dpf_gen_seeded(uint64_t alpha, uint32_t logN, const uint8_t s0[16], const uint8_t s1[16], uint8_t* ka,
                   uint8_t* kb);
/* Gen (dpf.go:71) itself: seeds from getrandom(2), like crypto/rand. */
int dpf_gen(uint64_t alpha, uint32_t logN, uint8_t* ka, uint8_t* kb);
/* n keys pairs at once over nthreads host threads (<= 0: all cores).
 * alphas[n], s0s/s1s [n][16], kas/kbs [n][dpf_key_len]. */
int dpf_gen_batch_seeded(const uint64_t* alphas, uint32_t logN, const uint8_t* s0s, const uint8_t* s1s, size_t n,
                         uint8_t* kas, uint8_t* kbs, int nthreads);

/* ---- key wire format ------------------------------------ */
/* A key is the reference's DPFkey bytes (type DPFkey []byte, dpf.go:7; layout
 * dpf.go:89-92,111-112,137-138,165-167), so a key made by the Go Gen is a
 * valid input here and vice versa.  A batch is [n][key_len] contiguous (what
 * dpf_gen_batch_seeded writes and every batched entry reads).
 * dpf_keys_pack gathers n keys (pointers; lens[i] must equal key_len, or
 * lens = NULL) into out[n][key_len]: DPF_ERR_KEYLEN on a length mismatch.
 * dpf_keys_unpack scatters a batch back to n key buffers of key_len bytes.
 * Host-only; large batches are copied on several threads. */
int dpf_keys_pack(const uint8_t* const* keys, const size_t* lens, size_t n, size_t key_len, uint8_t* out);
int dpf_keys_unpack(const uint8_t* packed, size_t key_len, size_t n, uint8_t* const* keys);

/* ---- evaluation, host buffers (synchronous; PCIe-inclusive) ------------ */
/* Keys: at least 17 + 18*stop bytes (the reference's own index bound,
 * dpf.go:175-176,186-188); the final CW is always k[len-16 : len]
 * (dpf.go:206,219), longer keys are accepted.  Shorter: DPF_ERR_KEYLEN. */
/* Eval (dpf.go:171-211): *out_bit = 0/1.  Like the reference, Eval accepts
 * any logN (Gen never makes a key above 63): path bits above bit 63 of x read
 * as 0 (Go's `uint64(1) << s` is 0 for s >= 64, dpf.go:194), so such a key
 * takes the left child on its top logN-64 levels.  The EvalFull entry points
 * return DPF_ERR_PARAM for logN > 63, where the reference panics allocating
 * its 2^(logN-3)-byte output (dpf.go:251). */
int dpf_eval(const uint8_t* key, size_t key_len, uint64_t x, uint32_t logN, uint8_t* out_bit);
/* Host output buffers are written by parallel copies from pinned staging;
 * with DPF_PREFAULT_OUTPUT=1 in the environment, buffers >= 64 MiB also get
 * a MADV_HUGEPAGE hint and are pre-touched (zeroed) while the GPU works.
 * Off by default: it changes the caller's memory policy. */
/* EvalFull (dpf.go:243-262): out = dpf_evalfull_len(logN) bytes. */
int dpf_evalfull(const uint8_t* key, size_t key_len, uint32_t logN, uint8_t* out);
/* nkeys x EvalFull; keys packed [nkeys][key_len], out [nkeys][evalfull_len].
 * Keys are sharded over ngpus devices (<= 0: all opened devices). */
int dpf_evalfull_batch(const uint8_t* keys, size_t key_len, size_t nkeys, uint32_t logN, uint8_t* out, int ngpus);
/* nkeys x pts_per_key Eval; xs [nkeys][pts_per_key], out one 0/1 byte per
 * query in the same order. */
int dpf_eval_batch(const uint8_t* keys, size_t key_len, size_t nkeys, const uint64_t* xs, size_t pts_per_key,
                   uint32_t logN, uint8_t* out, int ngpus);
/* One EvalFull split by top-level subtree over ngpus devices (ngpus must be
 * a power of two <= 2^stop); out = dpf_evalfull_len(logN) bytes. */
int dpf_evalfull_split(const uint8_t* key, size_t key_len, uint32_t logN, uint8_t* out, int ngpus);

/* ---- evaluation, device-resident buffers (asynchronous on `stream`) ----
 * Pointers are device pointers on `device`; `work` holds
 * dpf_workspace_size(nkeys, logN) bytes; stream is a hipStream_t (NULL =
 * the default stream).  Nothing is synchronised. */
int dpf_evalfull_batch_dev(int device, const uint8_t* d_keys, size_t key_len, size_t nkeys, uint32_t logN,
                           uint8_t* d_out, void* d_work, void* stream);
/* The subtree at depth prefix_bits, index prefix of every key: 2^(logN-3-
 * prefix_bits) bytes per key at d_out + k*that (logN-7 >= prefix_bits). */
int dpf_evalfull_subtree_dev(int device, const uint8_t* d_keys, size_t key_len, size_t nkeys, uint32_t logN,
                             uint32_t prefix_bits, uint64_t prefix, uint8_t* d_out, void* d_work, void* stream);
/* Batched Eval on HBM buffers.  d_work holds work_bytes; with
 * dpf_eval_workspace_size(nkeys, pts_per_key, logN) bytes the queries of a
 * key share its top tree levels (a frontier of 2^L nodes per key computed
 * once); with only dpf_workspace_size(nkeys, logN) bytes each query walks
 * from the root.  Results are identical either way.  d_xs must be 8-byte
 * aligned (DPF_ERR_PARAM otherwise); a 16-byte-aligned d_xs lets the
 * persistent kernel stage query pairs by LDS-DMA, an 8-byte-aligned one
 * (e.g. a tensor slice xs[1:]) runs the per-pair kernel, same results. */
size_t dpf_eval_workspace_size(size_t nkeys, size_t pts_per_key, uint32_t logN);
/* Depth L of that shared frontier (0: none).  Work with the frontier:
 * 2^(L+1)-2 AES per key for the frontier nodes, then logN-7-L+1 per query
 * (against the reference's 2*(logN-7)+1, dpf.go:183-209). */
uint32_t dpf_eval_frontier_level(uint32_t logN, size_t pts_per_key);
int dpf_eval_batch_dev(int device, const uint8_t* d_keys, size_t key_len, size_t nkeys, const uint64_t* d_xs,
                       size_t pts_per_key, uint32_t logN, uint8_t* d_out, void* d_work, size_t work_bytes,
                       void* stream);

/* ---- CU-partitioned streams (no reference counterpart: engine plumbing) -
 * A stream whose kernels may run only on CUs [cu_first, cu_first+cu_count)
 * of `device` (hipExtStreamCreateWithCUMask).  Bit i of the mask is spread
 * across the XCDs (consecutive bits land on different XCDs), so any
 * contiguous range is balanced over the chip.  The _dev entry points size
 * their grids to the stream's CUs.  Two such streams over disjoint ranges let
 * an LDS-bound kernel (the tree) and an HBM-bound one (the PIR fold) run side
 * by side without sharing a CU.  Destroy with dpf_stream_destroy. */
int dpf_stream_create_cu_masked(int device, uint32_t cu_first, uint32_t cu_count, void** stream);
int dpf_stream_destroy(void* stream);

/* ---- AES back end of the tree kernels (BASELINE configs[1]) ------------
 * DPF_AES_TTABLE: T-tables staged in LDS (aes_ttable.hpp).
 * DPF_AES_BITSLICED: table-free byte-sliced AES, 8 blocks per lane in VALU
 * registers (aes_bytesliced.hpp); used for EvalFull subtrees of >= 2^7 leaf
 * blocks per key, the T-table elsewhere.  Outputs are bit-identical.
 * Process-wide; the default comes from env DPF_AES_IMPL=ttable|bitsliced. */
#define DPF_AES_TTABLE 0
#define DPF_AES_BITSLICED 1
int dpf_set_aes_impl(int impl);   /* returns the previous back end */
int dpf_get_aes_impl(void);
/* ---- batched Eval kernel (dpf_eval_batch*, BASELINE configs[2]) ---------
 * DPF_EVAL_WALK (default): the level-L frontier, then one walk per query.
 * DPF_EVAL_TRIE: the same frontier, then only the visited nodes of each
 * key's query trie below it (5,307 instead of 6,142 AES per
 * key at configs[2]), where logN <= 20 and pts_per_key <= 1024; the walk
 * kernel elsewhere.  Outputs are bit-identical.  The trie kernel was
 * measured slower and is built only in the experimental library (make
 * -C dpf-go_amd experimental); the product library returns DPF_ERR_PARAM
 * for DPF_EVAL_TRIE.  Process-wide; env DPF_EVAL_TRIE=1 sets the initial
 * value (experimental build). */
#define DPF_EVAL_WALK 0
#define DPF_EVAL_TRIE 1
int dpf_set_eval_kernel(int kernel);   /* returns the previous kernel */
int dpf_get_eval_kernel(void);
/* ---- small-call path of the single-key API ---------------
 * dpf_eval and dpf_evalfull are the reference's latency-bound single calls
 * (dpf.go:171, :243).  DPF_SMALL_AUTO (default) evaluates them on the host's
 * AES units (host_eval.cpp: AES-NI/VAES, bit-exact with the kernels) when
 * that beats a GPU round trip: every dpf_eval, and dpf_evalfull up to
 * logN = dpf_small_call_max_logN(), which depends on the host (21 with
 * VAES, 20 with AES-NI only); DPF_SMALL_GPU always uses the GPU,
 * DPF_SMALL_HOST the host whenever it has AES-NI, except dpf_evalfull above
 * logN = 28 (outputs of 32 MiB and more), which stays on the GPU.  Either
 * way a gfx950
 * device must be open (DPF_ERR_NODEV otherwise): this is a latency path,
 * not a fallback.  The batched and _dev entry points always run on the GPU.
 * Process-wide; default from env DPF_SMALL_CALLS=auto|gpu|host. */
#define DPF_SMALL_AUTO 0
#define DPF_SMALL_GPU 1
#define DPF_SMALL_HOST 2
int dpf_set_small_call_path(int mode);   /* returns the previous mode */
int dpf_get_small_call_path(void);
uint32_t dpf_small_call_max_logN(void);
/* aes128MMO (aes_amd64.s:51-82) of nblocks (multiple of 8) 16-byte blocks,
 * iterated `reps` times (out = MMO^reps(in)), under the fixed left (right=0)
 * or right key (dpf.go:23-24): the AES blocks/s microbenchmark + self-test. */
int dpf_aes_mmo_dev(int device, int impl, int right, const uint8_t* d_in, uint8_t* d_out, size_t nblocks,
                    uint32_t reps, void* stream);

/* Two-phase form of the above: expand keys once into d_work (the aligned
 * per-level records the kernels read), then evaluate any number of
 * subtrees of all nkeys keys from the expanded form.  Lets a caller time the
 * tree kernel alone and reuse expanded keys across calls.  The layout
 * depends on (nkeys, logN): dpf_evalfull_expanded_dev must pass the nkeys
 * and logN that dpf_expand_keys_dev used for this d_work, else
 * DPF_ERR_PARAM.  d_work is also the byte-sliced back end's frontier
 * scratch, so evaluations from one d_work must not overlap in time (use
 * one d_work per stream). */
int dpf_expand_keys_dev(int device, const uint8_t* d_keys, size_t key_len, size_t nkeys, uint32_t logN, void* d_work,
                        void* stream);
int dpf_evalfull_expanded_dev(int device, void* d_work, size_t nkeys, uint32_t logN, uint32_t prefix_bits,
                              uint64_t prefix, uint8_t* d_out, void* stream);
/* The library remembers, per d_work address, what dpf_expand_keys_dev (and
 * the other _dev entry points that expand into a caller's workspace) left
 * there.  Call this before freeing a workspace: a new buffer later allocated
 * at the same address would otherwise pass dpf_evalfull_expanded_dev's
 * shape check with stale records.  Always returns 0. */
int dpf_forget_workspace(const void* d_work);

/* ---- 2-server PIR over a DPF (BASELINE configs[4]; no reference
 *      counterpart: a consumer of EvalFull, SURVEY 8a last row) -----------
 * Server answer for key k: XOR of the 32-byte records DB[i] with
 * bit i of EvalFull(key_k, logN) set.  The DB holds nrec <= 2^logN records
 * of 32 bytes; the two servers' answers XOR to DB[alpha]. */

/* Device form on one GPU: DB slice = records of subtree (prefix_bits,
 * prefix), i.e. global records [prefix*2^(logN-prefix_bits), ...), d_db
 * holding nrec <= 2^(logN-prefix_bits) of them.  d_ans = nkeys*32 bytes
 * (overwritten); d_work = dpf_pir_workspace_size(nkeys, logN, prefix_bits). */
size_t dpf_pir_workspace_size(size_t nkeys, uint32_t logN, uint32_t prefix_bits);
int dpf_pir_answer_dev(int device, const uint8_t* d_keys, size_t key_len, size_t nkeys, uint32_t logN,
                       uint32_t prefix_bits, uint64_t prefix, const uint8_t* d_db, uint64_t nrec, uint8_t* d_ans,
                       void* d_work, void* stream);

/* Streaming consumer of EvalFull output, the PIR fold
 * generalised to any payload: for each key k,
 *   ans[k] = XOR over i < nrec with bit i of bits[k] set of payload[i]
 * (bit i = bit i%8 of byte i/8, EvalFull's layout, dpf.go:251-261), computed
 * where the EvalFull output already lives, so it never leaves HBM.
 * d_bits [nkeys][bits_stride] (e.g. dpf_evalfull_batch_dev's output;
 * bits_stride a multiple of 16, nrec <= 8*bits_stride), d_payload
 * [nrec][rec_bytes] (rec_bytes a positive multiple of 32), d_ans
 * [nkeys][rec_bytes] (overwritten), d_work dpf_xor_fold_workspace_size()
 * bytes; 16-byte-aligned device pointers.  Asynchronous on `stream`. */
size_t dpf_xor_fold_workspace_size(void);
int dpf_xor_fold_dev(int device, const uint8_t* d_bits, size_t bits_stride, size_t nkeys, const uint8_t* d_payload,
                     uint64_t nrec, size_t rec_bytes, uint8_t* d_ans, void* d_work, void* stream);

/* The fold on the matrix cores (v_mfma_scale_f32_32x32x64_f8f6f4, FP4 {0,1}
 * operands, exact counts whose parity is the answer bit) reads the DB in a
 * bit-sliced layout that a PIR server builds once when it loads the DB:
 * dbs[S][n][g] (u32) for super-group S of 256 records, bit position n < 256
 * and record group g < 8, bit j = bit n of record 256*S + 32*g + j (records
 * past nrec read as 0).  dpf_pir_db_slice_dev writes it from the row-major
 * DB (nrec x 32 B) into dpf_pir_db_sliced_size(nrec) bytes.  The _sliced
 * entry points take that layout and give the same answers as their row-major
 * forms (same workspace sizes); 32-byte records only. */
size_t dpf_pir_db_sliced_size(uint64_t nrec);
int dpf_pir_db_slice_dev(int device, const uint8_t* d_db, uint64_t nrec, uint8_t* d_dbs, void* stream);
int dpf_pir_answer_sliced_dev(int device, const uint8_t* d_keys, size_t key_len, size_t nkeys, uint32_t logN,
                              uint32_t prefix_bits, uint64_t prefix, const uint8_t* d_dbs, uint64_t nrec,
                              uint8_t* d_ans, void* d_work, void* stream);
int dpf_xor_fold_sliced_dev(int device, const uint8_t* d_bits, size_t bits_stride, size_t nkeys, const uint8_t* d_dbs,
                            uint64_t nrec, uint8_t* d_ans, void* d_work, void* stream);
/* Tuning / test limits of the XOR fold launches (process-wide; 0 = default):
 * at most max_blocks workgroups per fold launch (default and maximum 1024),
 * and at most max_sg_per_block super-groups of 256 records per matrix-core
 * fold workgroup (default and maximum 2^15).  The matrix-core fold's answer
 * bits are parities of fp32 counts, exact up to 2^24; with at most 2^23
 * records per workgroup no count gets there, and a DB with more super-groups
 * than max_blocks x max_sg_per_block is folded in passes.  Answers do not
 * depend on either; tests use them to force multi-pass folds.  Returns 0. */
int dpf_set_fold_limits(uint32_t max_blocks, uint32_t max_sg_per_block);
/* Kernel shape of dpf_pir_answer_sliced_dev (and of a sliced PIR handle):
 * DPF_PIR_SPLIT (default): a tree launch writes the selection bits to HBM
 * and a fold launch reads them back.  DPF_PIR_FUSED: where nkeys <= 64 and
 * the slice holds 2^8..2^10 blocks of 256 leaf pairs (logN - prefix_bits =
 * 24..26), one launch runs the subtree EvalFull and the matrix-core fold
 * together (k_pir_fused: per CU, 12 waves expand the tree with one key per
 * lane and 4 waves fold each leaf pair from LDS), so the selection bits
 * never reach HBM; measured slower on MI355X, the split
 * path elsewhere.  DPF_PIR_FUSED_ANY fuses any slice from logN -
 * prefix_bits = 16 (test mode).  Answers are identical.  The fused kernel is
 * built only in the experimental library (make -C dpf-go_amd experimental):
 * the product library returns DPF_ERR_PARAM for DPF_PIR_FUSED and
 * DPF_PIR_FUSED_ANY.  Process-wide; env DPF_PIR_KERNEL=split|fused|fused-any. */
#define DPF_PIR_SPLIT 0
#define DPF_PIR_FUSED 1
#define DPF_PIR_FUSED_ANY 2
int dpf_set_pir_kernel(int kernel);   /* returns the previous kernel */
int dpf_get_pir_kernel(void);
/* What dpf_pir_answer_sliced_dev runs for this shape under the current
 * setting and AES back end: DPF_PIR_FUSED or DPF_PIR_SPLIT. */
int dpf_pir_kernel_for(size_t nkeys, uint32_t logN, uint32_t prefix_bits);

/* Host form: the DB is uploaded once, sharded by top-level subtree over
 * ngpus devices (a power of two), each GPU folds its slice and the host
 * XORs the per-GPU partial answers (RCCL has no XOR reduction). */
int dpf_pir_db_create(const uint8_t* db, uint64_t nrec, uint32_t logN, int ngpus, void** handle);
int dpf_pir_answer(void* handle, const uint8_t* keys, size_t key_len, size_t nkeys, uint8_t* ans);
void dpf_pir_db_free(void* handle);

#ifdef __cplusplus
}
#endif

#endif /* DPF_HIP_H */
