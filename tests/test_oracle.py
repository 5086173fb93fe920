"""CPU tests: the oracle against independent pins (OpenSSL AES KATs, the
reference's own property tests dpf/dpf_test.go:32-73) and the committed
golden vectors."""
import hashlib
import json
import os

import numpy as np
import pytest

import oracle

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _load(name):
    with open(os.path.join(GOLD, name)) as f:
        return json.load(f)


def test_aes_fips197():
    kat = _load("aes_kat.json")["fips197_c1"]
    assert oracle.aes128_encrypt(bytes.fromhex(kat["key"]), bytes.fromhex(kat["pt"])).hex() == kat["ct"]


@pytest.mark.parametrize("aesni", [False, True])
def test_fixed_key_mmo_kat(aesni):
    if aesni and not oracle.have_aesni():
        pytest.skip("no AES-NI on this host")
    kat = _load("aes_kat.json")
    kl = bytes.fromhex(kat["fixed_keys"]["keyL"])
    kr = bytes.fromhex(kat["fixed_keys"]["keyR"])
    for v in kat["vectors"]:
        pt = bytes.fromhex(v["pt"])
        assert oracle.aes128_encrypt(kl, pt).hex() == v["aes_L"]
        assert oracle.aes128_encrypt(kr, pt).hex() == v["aes_R"]
        assert oracle.mmo(False, pt, aesni).hex() == v["mmo_L"]
        assert oracle.mmo(True, pt, aesni).hex() == v["mmo_R"]


def _bits(b: bytes) -> np.ndarray:
    return np.unpackbits(np.frombuffer(b, np.uint8), bitorder="little")


# Restatement of TestEval (dpf_test.go:32-43): Eval(ka,x)^Eval(kb,x) == [x==alpha].
@pytest.mark.parametrize("trial", range(3))
def test_reference_TestEval(trial):
    logN, alpha = 8, 123
    rng = np.random.default_rng(trial)
    ka, kb = oracle.gen(alpha, logN, rng.bytes(16), rng.bytes(16))
    for i in range(1 << logN):
        assert (oracle.eval_(ka, i, logN) ^ oracle.eval_(kb, i, logN)) == (1 if i == alpha else 0)


# TestEvalFull (dpf_test.go:45-58) and TestEvalFullShort (:60-73).
@pytest.mark.parametrize("logN,alpha", [(9, 128), (3, 1)])
@pytest.mark.parametrize("trial", range(3))
def test_reference_TestEvalFull(logN, alpha, trial):
    rng = np.random.default_rng(100 + trial)
    ka, kb = oracle.gen(alpha, logN, rng.bytes(16), rng.bytes(16))
    a, b = _bits(oracle.evalfull(ka, logN)), _bits(oracle.evalfull(kb, logN))
    x = (a ^ b)[: 1 << logN]
    assert x[alpha] == 1 and x.sum() == 1


@pytest.mark.parametrize("logN", [0, 1, 2, 5, 6, 7, 10, 14])
def test_share_xor_is_point_function(logN):
    rng = np.random.default_rng(logN)
    n = 1 << logN
    for alpha in sorted({0, n - 1, int(rng.integers(0, n))}):
        ka, kb = oracle.gen(alpha, logN, rng.bytes(16), rng.bytes(16))
        x = (_bits(oracle.evalfull(ka, logN)) ^ _bits(oracle.evalfull(kb, logN)))[:n]
        assert x[alpha] == 1 and x.sum() == 1
        for q in range(0, n, max(1, n // 64)):
            assert oracle.eval_(ka, q, logN) == _bits(oracle.evalfull(ka, logN))[q]


def test_key_layout():
    for logN in (0, 6, 7, 20, 32, 63):
        stop = max(logN - 7, 0)
        assert oracle.key_len(logN) == 33 + 18 * stop
        assert oracle.out_len(logN) == (16 if logN < 7 else 1 << (logN - 3))
    with pytest.raises(ValueError):
        oracle.gen(8, 3, bytes(16), bytes(16))
    with pytest.raises(ValueError):
        oracle.gen(0, 64, bytes(16), bytes(16))


def test_oracle_matches_golden():
    for c in _load("dpf_golden.json")["cases"]:
        logN = c["logN"]
        ka, kb = oracle.gen(c["alpha"], logN, bytes.fromhex(c["s0"]), bytes.fromhex(c["s1"]))
        assert ka.hex() == c["ka"] and kb.hex() == c["kb"]
        fa, fb = oracle.evalfull(ka, logN), oracle.evalfull(kb, logN)
        if "full_a" in c:
            assert fa.hex() == c["full_a"] and fb.hex() == c["full_b"]
        else:
            assert hashlib.sha256(fa).hexdigest() == c["full_a_sha256"]
            assert hashlib.sha256(fb).hexdigest() == c["full_b_sha256"]
        for x, ea, eb in zip(c["eval_xs"], c["eval_a"], c["eval_b"]):
            assert oracle.eval_(ka, x, logN) == ea and oracle.eval_(kb, x, logN) == eb


def test_aesni_and_portable_agree():
    if not oracle.have_aesni():
        pytest.skip("no AES-NI")
    rng = np.random.default_rng(7)
    keys = np.frombuffer(rng.bytes(6 * oracle.key_len(12)), np.uint8).reshape(6, -1)
    a = oracle.evalfull_batch(keys, 12, nthreads=3, aesni=True)
    b = np.stack([np.frombuffer(oracle.evalfull(k.tobytes(), 12, aesni=False), np.uint8) for k in keys])
    assert np.array_equal(a, b)


def test_oracle_threaded_evalfull_and_sliced_pir_match_restatement():
    """The threaded subtree EvalFull and the batched sliced PIR answer (used
    by the full-size GPU parity tests) equal the plain restatements."""
    import numpy as np
    from dpf import synth
    for logN in (7, 9, 14):
        al, s0, s1 = synth.key_seeds(2, logN, first=70 + logN)
        for i in range(2):
            ka, _ = oracle.gen(int(al[i]), logN, s0[i].tobytes(), s1[i].tobytes())
            for nt in (1, 3, 8):
                assert oracle.evalfull_mt(ka, logN, nt).tobytes() == oracle.evalfull(ka, logN)
    logN, nrec = 12, (1 << 12) - 77
    db = synth.db_bytes(nrec * 32).reshape(nrec, 32)
    al, s0, s1 = synth.key_seeds(4, logN, first=9)
    keys = np.stack([np.frombuffer(oracle.gen(int(al[i]), logN, s0[i].tobytes(), s1[i].tobytes())[0], np.uint8)
                     for i in range(4)])
    a = oracle.pir_answer_batch(keys, logN, db, nrec, nslices=8, nthreads=3)
    for i in range(4):
        assert np.bitwise_xor.reduce(a[i], axis=0).tobytes() == oracle.pir_answer(keys[i].tobytes(), logN, db, 0, nrec)
        for s in range(8):
            lo, hi = s << 9, min(nrec, (s + 1) << 9)
            assert a[i, s].tobytes() == oracle.pir_answer(keys[i].tobytes(), logN, db[lo:hi], lo, hi - lo)
