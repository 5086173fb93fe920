"""CPU tests of the product boundary: libdpf_hip.so loads and exports every
function include/dpf_hip.h declares, host-side Gen matches the golden keys,
parameter validation mirrors the reference's panics.  No GPU compute."""
import json
import os
import re

import numpy as np
import pytest

import dpf
from dpf import synth

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(ROOT, "tests", "golden")


def _header_functions():
    src = open(os.path.join(ROOT, "include", "dpf_hip.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(dpf_[A-Za-z0-9_]+)\s*\(", src)))


def test_library_exports_every_header_symbol():
    L = dpf.lib()
    names = _header_functions()
    assert len(names) >= 20
    for n in names:
        assert hasattr(L, n), f"libdpf_hip.so does not export {n}"
    assert set(names) == set(dpf.SIGNATURES), "Python signature table out of sync with the header"


def test_library_binds_every_symbol_now():
    """Every kernel's host stub and every internal function is defined in the
    library: a shared object links with undefined symbols, and the gap shows
    only when that path is first called (r05: a kernel template whose host
    stub the compiler dropped).  dlopen with RTLD_NOW resolves them all, and
    no undefined symbol of the library's own namespaces is left."""
    import ctypes
    import subprocess
    ctypes.CDLL(dpf.LIB_PATH, mode=os.RTLD_NOW | os.RTLD_LOCAL)
    out = subprocess.run(["nm", "-D", "--undefined-only", dpf.LIB_PATH], capture_output=True, text=True, check=True)
    own = [ln for ln in out.stdout.splitlines() if "dpfk" in ln or "dpfh" in ln or "dpfc" in ln]
    assert not own, own[:5]


def test_library_is_gfx950_code_object():
    blob = open(dpf.LIB_PATH, "rb").read()
    assert b"gfx950" in blob


def test_sizes():
    for logN in (0, 3, 6, 7, 8, 20, 32, 63):
        stop = max(logN - 7, 0)
        assert dpf.key_len(logN) == 33 + 18 * stop
        assert dpf.evalfull_len(logN) == (16 if logN < 7 else 1 << (logN - 3))
    # T-table records + byte-sliced CW words + byte-sliced frontier (up to 2^10 nodes x 17 B per key)
    al = lambda x: (x + 255) // 256 * 256
    assert dpf.workspace_size(4096, 20) == (al(4096 * (13 + 2) * 32) + al(4096 * (13 * 36 + 32) * 4)
                                            + al(4096 * 1024 * 17))


def test_host_gen_matches_golden():
    cases = json.load(open(os.path.join(GOLD, "dpf_golden.json")))["cases"]
    for c in cases:
        ka, kb = dpf.gen_seeded(c["alpha"], c["logN"], bytes.fromhex(c["s0"]), bytes.fromhex(c["s1"]))
        assert ka.hex() == c["ka"] and kb.hex() == c["kb"]


def test_key_pack_unpack_roundtrip():
    """Key wire format: a batch is [n][key_len] of the
    reference's DPFkey bytes; pack/unpack are exact inverses, also on the
    multi-threaded path (> 8 MiB)."""
    for logN, n in ((20, 1), (20, 300), (3, 5), (24, 30000)):
        al, s0, s1 = synth.key_seeds(n, logN)
        ka, _ = dpf.gen_batch_seeded(al, logN, s0, s1)
        keys = [bytes(k) for k in ka]
        packed = dpf.keys_pack(keys)
        assert packed.shape == (n, dpf.key_len(logN)) and np.array_equal(packed, ka)
        assert dpf.keys_unpack(packed) == keys
    assert dpf.keys_pack([]).shape == (0, 0)


def test_key_pack_rejects_ragged_batches():
    ka, kb = dpf.gen_seeded(5, 9, bytes(16), bytes(range(16)))
    with pytest.raises(dpf.DPFPanic) as e:
        dpf.keys_pack([ka, kb[:-1]])
    assert e.value.code == dpf.DPF_ERR_KEYLEN
    with pytest.raises(dpf.DPFPanic):
        dpf.keys_pack([ka], key_len=len(ka) + 1)


def test_xor_fold_validates_before_touching_a_device():
    """dpf_xor_fold_dev rejects bad shapes with DPF_ERR_PARAM (no GPU needed:
    validation precedes any device call); pointers are never dereferenced."""
    L = dpf.lib()
    p = 4096   # aligned fake device address, never used
    for stride, nrec, rec in ((16, 128, 48), (16, 128, 0), (24, 8, 32), (16, 129, 32)):
        assert L.dpf_xor_fold_dev(0, p, stride, 1, p, nrec, rec, p, p, None) == dpf.DPF_ERR_PARAM
    assert L.dpf_xor_fold_dev(0, p + 4, 16, 1, p, 128, 32, p, p, None) == dpf.DPF_ERR_PARAM   # misaligned bits
    assert dpf.xor_fold_workspace_size() > 0


def test_expanded_form_requires_an_expanded_workspace():
    """dpf_evalfull_expanded_dev refuses a d_work that dpf_expand_keys_dev did
    not expand for this (nkeys, logN): the records' layout depends on both
    (ADVICE r02).  Checked before any device call."""
    L = dpf.lib()
    p = 8192   # fake device address, never dereferenced
    assert L.dpf_evalfull_expanded_dev(0, p, 4, 20, 0, 0, p, None) == dpf.DPF_ERR_PARAM
    assert L.dpf_evalfull_expanded_dev(0, p, 0, 20, 0, 0, p, None) == dpf.DPF_OK   # no keys: nothing to do


def test_batch_gen_matches_single():
    logN = 20
    al, s0, s1 = synth.key_seeds(64, logN)
    ka, kb = dpf.gen_batch_seeded(al, logN, s0, s1, nthreads=4)
    for i in (0, 17, 63):
        a, b = dpf.gen_seeded(int(al[i]), logN, s0[i].tobytes(), s1[i].tobytes())
        assert ka[i].tobytes() == a and kb[i].tobytes() == b


def test_gen_random_keys_are_fresh_and_wellformed():
    ka, kb = dpf.Gen(123, 27)
    ka2, _ = dpf.Gen(123, 27)
    assert len(ka) == len(kb) == dpf.key_len(27)
    assert ka != ka2
    assert ka[16] ^ kb[16] == 1                       # t0 ^ t1 == 1 (dpf.go:83-84)
    assert ka[0] & 1 == 0 and kb[0] & 1 == 0          # seeds' LSB cleared (:86-87)
    assert ka[17:] == kb[17:]                         # shared CWs (:166-167)


@pytest.mark.parametrize("alpha,logN", [(8, 3), (1 << 20, 20), (0, 64), (5, 70)])
def test_gen_panics_like_reference(alpha, logN):
    with pytest.raises(dpf.DPFPanic) as e:
        dpf.Gen(alpha, logN)
    assert "invalid parameters" in str(e.value)
    with pytest.raises(dpf.DPFPanic):
        dpf.gen_seeded(alpha, logN, bytes(16), bytes(16))


def test_synth_is_deterministic():
    a = synth.key_seeds(8, 20)
    b = synth.key_seeds(8, 20)
    for x, y in zip(a, b):
        assert np.array_equal(x, y)
    assert int(a[0].max()) < (1 << 20)
    assert synth.eval_points(4, 16, 20).max() < (1 << 20)
    assert synth.db_bytes(100).shape == (100,)


def _build_c_smoke(tmp_path):
    """Compile tests/c/capi_smoke.c against include/dpf_hip.h with plain gcc
    (C99, -Werror): the header is C-clean and every symbol the program uses
    resolves from the shared library at link time."""
    import shutil
    import subprocess
    gcc = shutil.which("gcc") or shutil.which("cc")
    if gcc is None:
        pytest.skip("no C compiler")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    libdir = os.path.dirname(dpf.LIB_PATH)
    exe = str(tmp_path / "capi_smoke")
    subprocess.run([gcc, "-std=c99", "-O1", "-Wall", "-Werror", "-I", os.path.join(root, "include"),
                    os.path.join(root, "tests", "c", "capi_smoke.c"), "-o", exe, "-L", libdir, "-ldpf_hip",
                    "-Wl,-rpath," + libdir], check=True, capture_output=True, text=True)
    return exe


def test_c_program_links_against_header(tmp_path):
    assert os.path.exists(_build_c_smoke(tmp_path))


@pytest.mark.gpu
def test_c_program_runs_on_gpu(tmp_path):
    """The same checks as the reference's dpf_test.go, from C through the ABI."""
    import subprocess
    exe = _build_c_smoke(tmp_path)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "all checks passed" in r.stdout


def _asan_driver(tmp_path, build_lib: bool):
    """tests/c/host_sanity.c linked against the host-ASan/UBSan build of the
    library (`make -C dpf-go_amd asan`; sanitizers on host code only)."""
    import glob
    import subprocess
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    pkg = os.path.join(root, "dpf-go_amd")
    libdir = os.path.join(pkg, "lib", "asan")
    if build_lib:
        subprocess.run(["make", "-s", "-j4", "-C", pkg, "asan"], check=True, capture_output=True, text=True)
    if not os.path.exists(os.path.join(libdir, "libdpf_hip.so")):
        pytest.skip("ASan library not built (make -C dpf-go_amd asan)")
    clang = "/opt/rocm/lib/llvm/bin/clang"
    rt = glob.glob("/opt/rocm/lib/llvm/lib/clang/*/lib/linux/libclang_rt.asan-x86_64.so")
    if not os.path.exists(clang) or not rt:
        pytest.skip("no clang ASan runtime")
    exe = str(tmp_path / "host_sanity")
    subprocess.run([clang, "-std=c99", "-O1", "-g", "-Wall", "-Werror", "-fsanitize=address,undefined",
                    "-fno-omit-frame-pointer", "-shared-libasan", "-I", os.path.join(root, "include"),
                    os.path.join(root, "tests", "c", "host_sanity.c"), "-o", exe, "-L", libdir, "-ldpf_hip",
                    "-Wl,-rpath," + libdir, "-lpthread"], check=True, capture_output=True, text=True)
    env = dict(os.environ)
    env["LD_LIBRARY_PATH"] = os.path.dirname(rt[0]) + ":" + env.get("LD_LIBRARY_PATH", "")
    return exe, env


def test_host_sanitizers(tmp_path):
    """ASan (with leak detection) + UBSan over Gen, argument validation,
    no-device error paths and open/shutdown cycles of the host library."""
    import subprocess
    exe, env = _asan_driver(tmp_path, build_lib=True)
    env["ASAN_OPTIONS"] = "detect_leaks=1:abort_on_error=0"
    r = subprocess.run([exe], capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, r.stdout + r.stderr[-4000:]
    assert "host_sanity ok" in r.stdout


@pytest.mark.gpu
def test_host_sanitizers_with_gpu(tmp_path):
    """The same driver on the GPU box: concurrent host-buffer EvalFull/Eval
    from 4 threads racing shutdown/re-open, a PIR handle used and freed after
    shutdown, and a 2 MiB+ CopyPool copy, all under host ASan + UBSan (leak
    checking off: the HIP runtime keeps process-lifetime allocations)."""
    import subprocess
    exe, env = _asan_driver(tmp_path, build_lib=False)
    env["ASAN_OPTIONS"] = "detect_leaks=0:protect_shadow_gap=0"
    r = subprocess.run([exe, "gpu"], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stdout + r.stderr[-4000:]
    assert "host_sanity ok (gpu)" in r.stdout


# ---- host small-call path (host_eval.cpp) vs the oracle, no GPU needed ----
@pytest.fixture(scope="module")
def host_shim(tmp_path_factory):
    """tests/c/host_eval_shim.cpp linked with the library's host objects."""
    import ctypes
    import subprocess
    lib_dir = os.path.join(ROOT, "dpf-go_amd", "lib")
    objs = [os.path.join(lib_dir, o) for o in ("host_eval.o", "host_gen.o")]
    if not all(os.path.exists(o) for o in objs):
        pytest.skip("library not built (run __graft_entry__.build())")
    so = str(tmp_path_factory.mktemp("shim") / "libshim.so")
    subprocess.run(["g++", "-O2", "-shared", "-fPIC", "-o", so, os.path.join(ROOT, "tests", "c", "host_eval_shim.cpp"),
                    *objs, "-lpthread"], check=True)
    L = ctypes.CDLL(so)
    vp, sz = ctypes.c_void_p, ctypes.c_size_t
    L.shim_evalfull.argtypes = [vp, sz, ctypes.c_uint32, vp]
    L.shim_eval_batch.argtypes = [vp, sz, sz, vp, sz, ctypes.c_uint32, vp]
    if not L.shim_available():
        pytest.skip("no AES-NI on this host")
    return L


def _host_full(L, keys, logN):
    keys = np.ascontiguousarray(keys, np.uint8)
    out = np.zeros((keys.shape[0], dpf.evalfull_len(logN)), np.uint8)
    for k in range(keys.shape[0]):
        L.shim_evalfull(keys[k].ctypes.data, keys.shape[1], logN, out[k].ctypes.data)
    return out


def _host_eval(L, keys, xs, logN):
    keys = np.ascontiguousarray(keys, np.uint8)
    xs = np.ascontiguousarray(xs, np.uint64)
    out = np.zeros(xs.shape, np.uint8)
    L.shim_eval_batch(keys.ctypes.data, keys.shape[1], keys.shape[0], xs.ctypes.data, xs.shape[1], logN,
                      out.ctypes.data)
    return out


@pytest.mark.parametrize("isa", ["auto", "aesni"])
@pytest.mark.parametrize("logN", [0, 1, 3, 6, 7, 8, 9, 12, 15, 18, 20])
def test_host_path_matches_oracle(host_shim, logN, isa, monkeypatch):
    """Host EvalFull/Eval (VAES where the CPU has it, and the AES-NI form
    forced by DPF_HOST_ISA=aesni) are bit-exact with the oracle,
    dpf.go:171-262."""
    import oracle
    monkeypatch.setenv("DPF_HOST_ISA", isa)
    nk = 6 if logN < 18 else 2
    al, s0, s1 = synth.key_seeds(nk, logN, first=900 + logN)
    ka, kb = dpf.gen_batch_seeded(al, logN, s0, s1)
    keys = np.concatenate([ka, kb])
    assert np.array_equal(_host_full(host_shim, keys, logN), oracle.evalfull_batch(keys, logN, nthreads=4))
    xs = synth.eval_points(2 * nk, 37, logN)
    if logN < 7:
        xs[:, :5] = np.array([127, 128, 1000, 2 ** 40 + 3, 2 ** 64 - 1], np.uint64)   # x >= 2^logN: bit x & 127
    else:
        xs[:, :3] |= np.uint64(0xFFFF) << np.uint64(48)                                # ignored high bits
    assert np.array_equal(_host_eval(host_shim, keys, xs, logN), oracle.eval_batch(keys, xs, logN, nthreads=4))


@pytest.mark.parametrize("logN", [5, 9, 13])
def test_host_path_exactness_rules(host_shim, logN):
    """SURVEY §8c's rules on malformed keys: byte-valued t (not bit 0), an
    unmasked root LSB, the final CW at len-16 (also overlapping the last
    level record, and after extra trailing bytes)."""
    import oracle
    rng = np.random.default_rng(logN)
    stop = max(logN - 7, 0)
    al, s0, s1 = synth.key_seeds(4, logN, first=77)
    ka, _ = dpf.gen_batch_seeded(al, logN, s0, s1)
    cases = []
    k = ka[0].copy(); k[16] = 0x5A; k[0] |= 1
    cases.append(k)
    k = ka[1].copy()
    for i in range(stop):
        k[17 + 18 * i + 16: 17 + 18 * i + 18] = rng.integers(0, 256, 2, dtype=np.uint8)
    cases.append(k)
    cases.append(ka[2][: 17 + 18 * stop].copy())                                 # final CW overlaps the last record
    cases.append(np.concatenate([ka[3], rng.integers(0, 256, 9, dtype=np.uint8)]))   # trailing bytes
    for k in cases:
        k = k.reshape(1, -1)
        assert np.array_equal(_host_full(host_shim, k, logN), oracle.evalfull_batch(k, logN))
        xs = synth.eval_points(1, 64, logN)
        assert np.array_equal(_host_eval(host_shim, k, xs, logN), oracle.eval_batch(k, xs, logN))


def test_small_call_thresholds_match_the_recorded_crossovers():
    """the AUTO routing threshold of each host ISA is the largest
    logN at which the host EvalFull measured faster than the GPU round trip
    on the GPU box (tools/small_calls.py -> profiles/r05/small_calls), for
    VAES and for AES-NI only (DPF_HOST_ISA=aesni).  Checked against the
    recorded medians rather than a wall-clock race in the test, which the
    box's load would decide."""
    import subprocess
    import sys
    prof = os.path.join(ROOT, "profiles", "r05", "small_calls")
    flags = set()
    for ln in open("/proc/cpuinfo"):
        if ln.startswith("flags"):
            flags = set(ln.split(":", 1)[1].split())
            break
    if "aes" not in flags:
        pytest.skip("host without AES-NI")
    code = "import sys; sys.path.insert(0, %r); import dpf; print(dpf.small_call_max_logN())" % os.path.join(
        ROOT, "dpf-go_amd")
    for isa, name in (("aesni", "small_aesni.json"), ("auto", "small_vaes.json")):
        if isa == "auto" and not {"vaes", "avx512f"} <= flags:
            continue                                   # this CPU would take the AES-NI path
        rec = json.load(open(os.path.join(prof, name)))
        wins = sorted(int(n) for n, r in rec["evalfull"].items() if r["host_ms"] < r["gpu_ms"])
        losses = sorted(int(n) for n, r in rec["evalfull"].items() if r["host_ms"] >= r["gpu_ms"])
        assert wins and losses and max(wins) < min(losses), rec["evalfull"]
        env = dict(os.environ)
        env.pop("DPF_HOST_ISA", None)
        if isa == "aesni":
            env["DPF_HOST_ISA"] = "aesni"
        out = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, check=True)
        assert int(out.stdout.strip().splitlines()[-1]) == max(wins), (isa, out.stdout, max(wins))
