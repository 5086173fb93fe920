"""The single-key API's small-call path (include/dpf_hip.h
DPF_SMALL_*): dpf_eval / dpf_evalfull on the host's AES units when that
beats a GPU round trip.  Bit-exact with the oracle (dpf.go:171-262) in every
mode, routed as documented, and never without an open GPU."""
import time

import numpy as np
import pytest

import dpf
from dpf import synth
import oracle

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    assert dpf.gpu_init(1) >= 1
    prev = dpf.get_small_call_path()
    yield
    dpf.set_small_call_path(prev)


@pytest.mark.parametrize("mode", ["host", "auto", "gpu"])
@pytest.mark.parametrize("logN", [3, 7, 12, 20, 22])
def test_single_calls_match_oracle(mode, logN):
    dpf.set_small_call_path(mode)
    al, s0, s1 = synth.key_seeds(2, logN, first=5000 + logN)
    ka, kb = dpf.gen_batch_seeded(al, logN, s0, s1)
    for k in (ka[0], kb[1]):
        assert dpf.EvalFull(k.tobytes(), logN) == oracle.evalfull(k.tobytes(), logN, aesni=True)
        for x in list(synth.eval_points(1, 6, logN)[0]) + [int(al[0]), (1 << 63) | 5]:
            assert dpf.Eval(k.tobytes(), int(x), logN) == oracle.eval_(k.tobytes(), int(x), logN, aesni=True)


def test_two_server_property_through_the_host_path():
    dpf.set_small_call_path("host")
    logN = 16
    al, s0, s1 = synth.key_seeds(3, logN, first=61)
    ka, kb = dpf.gen_batch_seeded(al, logN, s0, s1)
    for j in range(3):
        x = np.frombuffer(dpf.EvalFull(ka[j].tobytes(), logN), np.uint8) ^ \
            np.frombuffer(dpf.EvalFull(kb[j].tobytes(), logN), np.uint8)
        bits = np.unpackbits(x, bitorder="little")
        assert bits.sum() == 1 and bits[int(al[j])] == 1


def test_short_key_still_panics_like_the_reference():
    dpf.set_small_call_path("host")
    with pytest.raises(dpf.DPFPanic) as e:
        dpf.EvalFull(bytes(40), 20)
    assert e.value.code == dpf.DPF_ERR_KEYLEN


def test_auto_mode_is_faster_than_the_gpu_round_trip_where_it_routes():
    """Loose sanity of the threshold: at logN = small_call_max_logN() the
    host call is not far slower than the GPU round trip (median of 15).  The
    threshold itself is measured by tools/small_calls.py for both host ISAs,
    and the CPU test test_capi.py::test_small_call_thresholds_match_the_
    recorded_crossovers holds the library to those measurements; a tight
    wall-clock ratio here would be at the mercy of host load and GPU clocks."""
    logN = dpf.small_call_max_logN()
    al, s0, s1 = synth.key_seeds(1, logN, first=9)
    ka, _ = dpf.gen_batch_seeded(al, logN, s0, s1)
    key = ka[0].tobytes()

    def med(mode):
        dpf.set_small_call_path(mode)
        dpf.EvalFull(key, logN)
        ts = []
        for _ in range(15):
            t0 = time.perf_counter()
            dpf.EvalFull(key, logN)
            ts.append(time.perf_counter() - t0)
        return float(np.median(ts))

    host, gpu = med("host"), med("gpu")
    assert host <= gpu * 5.0, (host, gpu)


@pytest.mark.parametrize("logN", [64, 65, 71, 90])
def test_eval_above_logN_63_like_the_reference(logN):
    """The reference's Eval validates no logN (dpf.go:171-211): with a long
    enough key it walks logN-7 levels, and `uint64(1) << (logN-1-i)` is 0 for
    shifts >= 64 (dpf.go:194), so the top logN-64 levels go left.  Gen cannot
    make such a key, so the keys are random bytes.  Host path, GPU single
    call and the batched kernel (root walks: no frontier above 63) all match
    the oracle; EvalFull rejects the logN like the reference's makeslice
    panic (dpf.go:251)."""
    rng = np.random.default_rng(logN)
    kl = 17 + 18 * (logN - 7) + 16
    keys = rng.integers(0, 256, size=(3, kl), dtype=np.uint8)
    keys[:, 16] = [0, 1, 7]                      # t bytes, byte-valued (dpf.go:176,185)
    xs = rng.integers(0, 2 ** 63, size=(3, 8), dtype=np.uint64) * np.uint64(2) + np.uint64(1)
    xs[:, 0] = 0
    xs[:, 1] = np.uint64(0xFFFFFFFFFFFFFFFF)
    want = oracle.eval_batch(keys, xs, logN, nthreads=1, aesni=True)
    for mode in ("host", "gpu"):
        dpf.set_small_call_path(mode)
        got = [[dpf.Eval(keys[k].tobytes(), int(x), logN) for x in xs[k]] for k in range(3)]
        assert np.array_equal(np.array(got, np.uint8), want), mode
    assert np.array_equal(dpf.eval_batch(keys, xs, logN, ngpus=1), want)
    assert dpf.eval_frontier_level(logN, 1 << 12) == 0
    with pytest.raises(dpf.DPFPanic) as e:
        dpf.EvalFull(keys[0].tobytes(), logN)
    assert e.value.code == dpf.DPF_ERR_PARAM
