#!/usr/bin/env python3
"""Regenerates the committed parity fixtures in tests/golden/.

  aes_kat.json   AES-128 known answers computed with the OpenSSL CLI
                 (`openssl enc -aes-128-ecb -nopad`), independent of any code
                 in this repo: FIPS-197 C.1 plus the two fixed PRG keys of
                 dpf/dpf.go:23-24 on several plaintexts, and the MMO values
                 (AES(x) ^ x, dpf/aes_amd64.s:79-80) derived from them.
  dpf_golden.json  DPF keys from the seeded Gen restatement (oracle/
                 dpf_oracle.c, following dpf/dpf.go:71-169 with s0/s1 fixed)
                 and their EvalFull / Eval outputs (hex, or SHA-256 when the
                 output exceeds 4 KiB), at logN in {0,1,2,3,6,7,8,9,13,20}
                 with alpha at the domain edges and leaf boundaries.

The reference itself (Go) cannot be run in this image; the oracle these
vectors come from is pinned by aes_kat.json and by the reference's three
property tests (dpf/dpf_test.go:32-73), which tests/test_oracle.py restates.
"""
from __future__ import annotations

import hashlib
import json
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "dpf-go_amd"))

KEY_L = bytes([36, 156, 50, 234, 92, 230, 49, 9, 174, 170, 205, 160, 98, 236, 29, 243])
KEY_R = bytes([209, 12, 199, 173, 29, 74, 44, 128, 194, 224, 14, 44, 2, 201, 110, 28])


def openssl_aes(key: bytes, pt: bytes) -> bytes:
    r = subprocess.run(["openssl", "enc", "-aes-128-ecb", "-nopad", "-K", key.hex()], input=pt,
                       capture_output=True, check=True)
    return r.stdout


def make_aes_kat() -> dict:
    pts = [bytes(16), bytes.fromhex("00112233445566778899aabbccddeeff"), bytes([0xff] * 16),
           bytes(range(16)), bytes.fromhex("80000000000000000000000000000001")]
    fips_key = bytes.fromhex("000102030405060708090a0b0c0d0e0f")
    out = {"source": "openssl enc -aes-128-ecb -nopad (OpenSSL CLI in the build image)",
           "fips197_c1": {"key": fips_key.hex(), "pt": pts[1].hex(), "ct": openssl_aes(fips_key, pts[1]).hex()},
           "fixed_keys": {"keyL": KEY_L.hex(), "keyR": KEY_R.hex()},
           "vectors": []}
    for pt in pts:
        cl = openssl_aes(KEY_L, pt)
        cr = openssl_aes(KEY_R, pt)
        out["vectors"].append({"pt": pt.hex(), "aes_L": cl.hex(), "aes_R": cr.hex(),
                               "mmo_L": bytes(a ^ b for a, b in zip(cl, pt)).hex(),
                               "mmo_R": bytes(a ^ b for a, b in zip(cr, pt)).hex()})
    return out


CASES = [  # (logN, [alphas])
    (0, [0]), (1, [0, 1]), (2, [3]), (3, [1, 7]), (6, [0, 63]), (7, [0, 127]), (8, [123, 128]),
    (9, [128, 511]), (13, [0, 127, 128, 8191]), (20, [0, 127, 128, (1 << 20) - 1, 0x5EED5]),
]


def make_dpf_golden() -> dict:
    import oracle
    from dpf import synth
    rows = []
    case_id = 0
    for logN, alphas in CASES:
        for alpha in alphas:
            _, s0, s1 = synth.key_seeds(1, 64, first=1000 + case_id)
            case_id += 1
            ka, kb = oracle.gen(alpha, logN, s0[0].tobytes(), s1[0].tobytes())
            fa, fb = oracle.evalfull(ka, logN), oracle.evalfull(kb, logN)
            n = 1 << logN
            xs = sorted({0, n - 1, alpha, alpha ^ 1 if (alpha ^ 1) < n else 0, (alpha + 128) % n,
                         (alpha * 7 + 3) % n, min(127, n - 1)})
            row = {"logN": logN, "alpha": alpha, "s0": s0[0].tobytes().hex(), "s1": s1[0].tobytes().hex(),
                   "ka": ka.hex(), "kb": kb.hex(),
                   "eval_xs": xs,
                   "eval_a": [oracle.eval_(ka, x, logN) for x in xs],
                   "eval_b": [oracle.eval_(kb, x, logN) for x in xs]}
            if len(fa) <= 4096:
                row["full_a"], row["full_b"] = fa.hex(), fb.hex()
            else:
                row["full_a_sha256"] = hashlib.sha256(fa).hexdigest()
                row["full_b_sha256"] = hashlib.sha256(fb).hexdigest()
            rows.append(row)
    return {"generator": "tests/golden/make_golden.py via oracle/dpf_oracle.c", "cases": rows}


def main() -> None:
    with open(os.path.join(HERE, "aes_kat.json"), "w") as f:
        json.dump(make_aes_kat(), f, indent=1)
    with open(os.path.join(HERE, "dpf_golden.json"), "w") as f:
        json.dump(make_dpf_golden(), f, indent=1)
    print("wrote aes_kat.json, dpf_golden.json")


if __name__ == "__main__":
    main()
