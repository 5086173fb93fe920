// Package dpf is the MI355X-backed drop-in for the evaluation path of
// github.com/dkales/dpf-go/dpf: the same exported API (DPFkey, Gen, Eval,
// EvalFull — reference dpf/dpf.go:7,71,171,243) over the C ABI of
// libdpf_hip.so (include/dpf_hip.h).  Gen stays on the host (AES-NI);
// Eval and EvalFull run as gfx950 kernels.  Where the reference panics,
// this package panics too.
//
// Build: make -C dpf-go_amd (produces dpf-go_amd/lib/libdpf_hip.so), then
// `go test ./...` in this directory on a machine with a gfx950 GPU.
package dpf

/*
#cgo CFLAGS: -I${SRCDIR}/../../../include
#cgo LDFLAGS: -L${SRCDIR}/../../lib -ldpf_hip -Wl,-rpath,${SRCDIR}/../../lib
#include <stdint.h>
#include "dpf_hip.h"
*/
import "C"

import (
	"crypto/rand"
	"unsafe"
)

// DPFkey is one party's key share, byte layout identical to the reference
// (dpf/dpf.go:89-167): seed[16] | t | per level (sCW[16] | tLCW | tRCW) | finalCW[16].
type DPFkey []byte

func check(rc C.int) {
	if rc != 0 {
		panic("dpf: " + C.GoString(C.dpf_last_error()))
	}
}

func u8(b []byte) *C.uint8_t {
	if len(b) == 0 {
		return nil
	}
	return (*C.uint8_t)(unsafe.Pointer(&b[0]))
}

// Gen mirrors dpf/dpf.go:71: two shares of the point function at alpha
// over a domain of 2^logN points; seeds come from crypto/rand (:80-81).
func Gen(alpha uint64, logN uint64) (DPFkey, DPFkey) {
	if alpha >= (1<<logN) || logN > 63 {
		panic("dpf: invalid parameters")
	}
	var seeds [32]byte
	if _, err := rand.Read(seeds[:]); err != nil {
		panic("dpf: crypto/rand failed")
	}
	n := int(C.dpf_key_len(C.uint32_t(logN)))
	ka := make(DPFkey, n)
	kb := make(DPFkey, n)
	check(C.dpf_gen_seeded(C.uint64_t(alpha), C.uint32_t(logN), u8(seeds[:16]), u8(seeds[16:]), u8(ka), u8(kb)))
	return ka, kb
}

// Eval mirrors dpf/dpf.go:171: this share's bit of f_alpha(x).
func Eval(k DPFkey, x uint64, logN uint64) byte {
	var out [1]byte
	check(C.dpf_eval(u8(k), C.size_t(len(k)), C.uint64_t(x), C.uint32_t(logN), u8(out[:])))
	return out[0]
}

// EvalFull mirrors dpf/dpf.go:243: this share of f_alpha over the whole
// domain, point x at bit x%8 of byte x/8 (16 bytes when logN < 7).
func EvalFull(key DPFkey, logN uint64) []byte {
	out := make([]byte, int(C.dpf_evalfull_len(C.uint32_t(logN))))
	check(C.dpf_evalfull(u8(key), C.size_t(len(key)), C.uint32_t(logN), u8(out)))
	return out
}

// EvalFullBatch evaluates many keys of one logN at once, sharded over
// ngpus GPUs (0 = all); out[i] is EvalFull(keys[i], logN).
func EvalFullBatch(keys []DPFkey, logN uint64, ngpus int) [][]byte {
	if len(keys) == 0 {
		return nil
	}
	kl := len(keys[0])
	packed := make([]byte, kl*len(keys))
	for i, k := range keys {
		if len(k) != kl {
			panic("dpf: keys of different lengths in one batch")
		}
		copy(packed[i*kl:], k)
	}
	ol := int(C.dpf_evalfull_len(C.uint32_t(logN)))
	flat := make([]byte, ol*len(keys))
	check(C.dpf_evalfull_batch(u8(packed), C.size_t(kl), C.size_t(len(keys)), C.uint32_t(logN), u8(flat),
		C.int(ngpus)))
	out := make([][]byte, len(keys))
	for i := range out {
		out[i] = flat[i*ol : (i+1)*ol : (i+1)*ol]
	}
	return out
}

// EvalBatch answers len(xs[i]) point queries for each key i.
func EvalBatch(keys []DPFkey, xs [][]uint64, logN uint64, ngpus int) [][]byte {
	if len(keys) == 0 {
		return nil
	}
	kl, ppk := len(keys[0]), len(xs[0])
	packed := make([]byte, kl*len(keys))
	pts := make([]uint64, ppk*len(keys))
	for i, k := range keys {
		if len(k) != kl || len(xs[i]) != ppk {
			panic("dpf: ragged batch")
		}
		copy(packed[i*kl:], k)
		copy(pts[i*ppk:], xs[i])
	}
	flat := make([]byte, ppk*len(keys))
	if ppk == 0 { // no queries: nothing to send (and &pts[0] would not exist)
		out := make([][]byte, len(keys))
		for i := range out {
			out[i] = flat[0:0:0]
		}
		return out
	}
	check(C.dpf_eval_batch(u8(packed), C.size_t(kl), C.size_t(len(keys)),
		(*C.uint64_t)(unsafe.Pointer(&pts[0])), C.size_t(ppk), C.uint32_t(logN), u8(flat), C.int(ngpus)))
	out := make([][]byte, len(keys))
	for i := range out {
		out[i] = flat[i*ppk : (i+1)*ppk : (i+1)*ppk]
	}
	return out
}

// PirDB is one PIR server's database of 32-byte records on the GPUs
// (dpf_pir_db_create): records are sharded over ngpus devices by top-level
// subtree, and Answer returns this server's 32-byte share per query key:
// the XOR of the records whose EvalFull bit is set (dpf.go:243-262).
type PirDB struct {
	h unsafe.Pointer
}

// NewPirDB uploads db (len(db)/32 records, at most 2^logN) to ngpus GPUs.
func NewPirDB(db []byte, logN uint64, ngpus int) *PirDB {
	if len(db)%32 != 0 {
		panic("dpf: PIR records are 32 bytes")
	}
	p := &PirDB{}
	var h unsafe.Pointer
	check(C.dpf_pir_db_create(u8(db), C.uint64_t(len(db)/32), C.uint32_t(logN), C.int(ngpus), &h))
	p.h = h
	return p
}

// Answer returns 32 bytes per key: keys[i]'s share of DB[alpha_i].
func (p *PirDB) Answer(keys []DPFkey) [][]byte {
	if len(keys) == 0 {
		return nil
	}
	kl := len(keys[0])
	packed := make([]byte, kl*len(keys))
	for i, k := range keys {
		if len(k) != kl {
			panic("dpf: keys of different lengths in one batch")
		}
		copy(packed[i*kl:], k)
	}
	flat := make([]byte, 32*len(keys))
	check(C.dpf_pir_answer(p.h, u8(packed), C.size_t(kl), C.size_t(len(keys)), u8(flat)))
	out := make([][]byte, len(keys))
	for i := range out {
		out[i] = flat[i*32 : (i+1)*32 : (i+1)*32]
	}
	return out
}

// Close frees the GPU copies of the database.
func (p *PirDB) Close() {
	if p.h != nil {
		C.dpf_pir_db_free(p.h)
		p.h = nil
	}
}

// Small-call routing of the single-key Eval / EvalFull (include/dpf_hip.h
// DPF_SMALL_*): SmallAuto (default) evaluates them on the host's AES units
// when that beats a GPU round trip, SmallGPU always uses the GPU, SmallHost
// the host whenever it has AES-NI.  A gfx950 device must be present in every
// mode.  Returns the previous mode.
const (
	SmallAuto = 0
	SmallGPU  = 1
	SmallHost = 2
)

func SetSmallCallPath(mode int) int {
	rc := C.dpf_set_small_call_path(C.int(mode))
	if rc < 0 {
		check(rc)
	}
	return int(rc)
}

// GetSmallCallPath returns the current small-call route (dpf_get_small_call_path).
func GetSmallCallPath() int {
	return int(C.dpf_get_small_call_path())
}

// SmallCallMaxLogN is the largest logN whose single-key EvalFull SmallAuto
// routes to the host (dpf_small_call_max_logN).
func SmallCallMaxLogN() uint64 {
	return uint64(C.dpf_small_call_max_logN())
}

// Batched Eval kernel (include/dpf_hip.h DPF_EVAL_*): EvalWalk (default)
// walks each query from the shared frontier, EvalTrie computes only the
// visited nodes of each key's query trie (logN <= 20, <= 1024 points per
// key; bit-identical, measured slower on MI355X; only in the experimental
// build, the product library panics on EvalTrie).  Returns the previous one.
const (
	EvalWalk = 0
	EvalTrie = 1
)

func SetEvalKernel(kernel int) int {
	rc := C.dpf_set_eval_kernel(C.int(kernel))
	if rc < 0 {
		check(rc)
	}
	return int(rc)
}

// GetEvalKernel returns the current batched Eval kernel (dpf_get_eval_kernel).
func GetEvalKernel() int {
	return int(C.dpf_get_eval_kernel())
}

// PIR kernel of the sliced PIR path (include/dpf_hip.h DPF_PIR_*): PirSplit
// (default) runs the tree launch then the fold launch, PirFused runs the
// subtree EvalFull and the matrix-core fold in one launch where it applies
// (<= 64 keys, logN - prefix_bits = 24..26; measured slower on MI355X),
// PirFusedAny fuses from logN - prefix_bits = 16 (test mode).  Answers are
// identical.  The fused kernel is only in the experimental build: the
// product library panics on PirFused / PirFusedAny.  Returns the previous one.
const (
	PirSplit    = 0
	PirFused    = 1
	PirFusedAny = 2
)

func SetPirKernel(kernel int) int {
	rc := C.dpf_set_pir_kernel(C.int(kernel))
	if rc < 0 {
		check(rc)
	}
	return int(rc)
}

// GetPirKernel returns the current PIR kernel setting (dpf_get_pir_kernel).
func GetPirKernel() int {
	return int(C.dpf_get_pir_kernel())
}

// SetFoldLimits caps the workgroups of a fold launch and the 256-record
// super-groups one matrix-core fold workgroup folds; larger DBs fold in
// passes (dpf_set_fold_limits; 0 = default).  Answers do not depend on
// either: tuning and tests only.
func SetFoldLimits(maxBlocks uint32, maxSgPerBlock uint32) {
	check(C.dpf_set_fold_limits(C.uint32_t(maxBlocks), C.uint32_t(maxSgPerBlock)))
}

// PirKernelFor reports which kernel a PIR answer of this shape runs now
// (dpf_pir_kernel_for): PirFused or PirSplit.
func PirKernelFor(nkeys int, logN uint64, prefixBits uint32) int {
	return int(C.dpf_pir_kernel_for(C.size_t(nkeys), C.uint32_t(logN), C.uint32_t(prefixBits)))
}
