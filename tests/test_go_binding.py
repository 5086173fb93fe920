"""The cgo package (dpf-go_amd/go/dpf) against the C ABI it binds, without Go.

Neither this container nor the GPU box has a Go toolchain (SURVEY §8c,
profiles/r04/round/go_probe.txt), so `go test` cannot run.  What
can be checked here is everything cgo itself would check at build time:

- every `C.dpf_*` call in the package names a function that include/dpf_hip.h
  declares and libdpf_hip.so exports;
- each call passes as many arguments as the prototype has parameters, and each
  argument's Go-side conversion (`C.size_t(...)`, `u8(...)`, `&h`, ...) is the
  C parameter's type (qualifiers aside);
- results wrapped in `check(...)` come from functions returning int (the Go
  wrapper panics on a nonzero code, as the reference panics, dpf/dpf.go:72-74);
- the cgo preamble compiles with gcc against the header and links against the
  library, taking the address of every bound function.

The package's own tests restate the reference's dpf/dpf_test.go:32-73; their C
twin runs on the GPU in tests/test_capi.py (tests/c/capi_smoke.c)."""
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GODIR = os.path.join(ROOT, "dpf-go_amd", "go", "dpf")
HEADER = os.path.join(ROOT, "include", "dpf_hip.h")
LIB = os.path.join(ROOT, "dpf-go_amd", "lib", "libdpf_hip.so")


def _strip_c_comments(s: str) -> str:
    s = re.sub(r"/\*.*?\*/", " ", s, flags=re.S)
    return re.sub(r"//[^\n]*", " ", s)


def _norm_type(t: str) -> str:
    t = t.replace("const", " ")
    t = re.sub(r"\s*\*\s*", "*", t)
    return re.sub(r"\s+", " ", t).strip()


def header_prototypes() -> dict:
    """{name: (return type, [parameter types])} for every dpf_* function."""
    src = _strip_c_comments(open(HEADER).read())
    src = re.sub(r"^\s*#.*$", " ", src, flags=re.M)
    protos = {}
    for m in re.finditer(r"([A-Za-z_][\w\s\*]*?)\b(dpf_\w+)\s*\(([^()]*)\)\s*;", src):
        ret, name, params = _norm_type(m.group(1)), m.group(2), m.group(3).strip()
        types = []
        if params and params != "void":
            for p in params.split(","):
                p = p.strip()
                arr = re.search(r"\[\s*\w*\s*\]\s*$", p)
                p = re.sub(r"\[\s*\w*\s*\]\s*$", "", p).strip()
                p = re.sub(r"\b\w+$", "", p).strip()          # drop the parameter name
                types.append(_norm_type(p) + ("*" if arr else ""))
        protos[name] = (ret, types)
    return protos


def _split_args(s: str) -> list:
    args, depth, cur = [], 0, ""
    for ch in s:
        if ch in "([{":
            depth += 1
        elif ch in ")]}":
            depth -= 1
        if ch == "," and depth == 0:
            args.append(cur.strip())
            cur = ""
        else:
            cur += ch
    if cur.strip():
        args.append(cur.strip())
    return args


def go_calls() -> list:
    """[(file, name, [argument expressions], wrapped_in_check)] for every C.dpf_* call."""
    calls = []
    for fn in sorted(os.listdir(GODIR)):
        if not fn.endswith(".go") or fn.endswith("_test.go"):
            continue
        src = open(os.path.join(GODIR, fn)).read()
        src = re.sub(r"//[^\n]*", "", src)
        for m in re.finditer(r"\bC\.(dpf_\w+)\(", src):
            i, depth = m.end(), 1
            while depth:
                depth += {"(": 1, ")": -1}.get(src[i], 0)
                i += 1
            before = src[max(0, m.start() - 6):m.start()]
            calls.append((fn, m.group(1), _split_args(src[m.end():i - 1]), before.endswith("check(")))
    return calls


def go_arg_type(expr: str):
    """The C type a Go argument expression converts to, or None if unknown."""
    m = re.fullmatch(r"C\.(\w+)\(.*\)", expr, flags=re.S)
    if m:
        return m.group(1)
    if re.fullmatch(r"u8\(.*\)", expr, flags=re.S):
        return "uint8_t*"
    m = re.fullmatch(r"\(\*C\.(\w+)\)\(.*\)", expr, flags=re.S)
    if m:
        return m.group(1) + "*"
    if expr == "&h":
        return "void**"
    if expr == "p.h":
        return "void*"
    return None


def test_go_package_present():
    calls = go_calls()
    assert calls, "no C.dpf_* calls found in the cgo package"
    names = {c[1] for c in calls}
    # the reference's exported API (dpf/dpf.go:71,171,243) and the PIR handle
    for need in ("dpf_gen_seeded", "dpf_eval", "dpf_evalfull", "dpf_evalfull_batch", "dpf_eval_batch",
                 "dpf_pir_db_create", "dpf_pir_answer", "dpf_pir_db_free", "dpf_last_error"):
        assert need in names, need


def test_every_bound_function_is_declared_with_matching_arguments():
    protos = header_prototypes()
    assert len(protos) > 40, "header parse found too few prototypes"
    for fn, name, args, checked in go_calls():
        assert name in protos, f"{fn}: C.{name} is not declared in include/dpf_hip.h"
        ret, params = protos[name]
        assert len(args) == len(params), f"{fn}: C.{name} takes {len(params)} arguments, the Go call passes {len(args)}"
        for i, (a, p) in enumerate(zip(args, params)):
            t = go_arg_type(a)
            assert t is not None, f"{fn}: C.{name} argument {i} ({a!r}) has no recognised cgo conversion"
            assert t == p, f"{fn}: C.{name} argument {i} ({a!r}) converts to {t}, the header wants {p}"
        if checked:
            assert ret == "int", f"{fn}: check(C.{name}(...)) but it returns {ret}"


def test_every_bound_function_is_exported():
    if not os.path.exists(LIB) or shutil.which("nm") is None:
        pytest.skip("libdpf_hip.so not built (make -C dpf-go_amd) or no nm")
    out = subprocess.run(["nm", "-D", "--defined-only", LIB], capture_output=True, text=True, check=True).stdout
    exported = {ln.split()[-1] for ln in out.splitlines() if ln.strip()}
    missing = sorted({n for _, n, _, _ in go_calls()} - exported)
    assert not missing, f"bound by the Go package but not exported by libdpf_hip.so: {missing}"


def test_cgo_preamble_compiles_and_links(tmp_path):
    gcc = shutil.which("gcc")
    if gcc is None or not os.path.exists(LIB):
        pytest.skip("gcc or libdpf_hip.so missing")
    src = open(os.path.join(GODIR, "dpf.go")).read()
    m = re.search(r"/\*(.*?)\*/\s*import \"C\"", src, flags=re.S)
    assert m, "no cgo preamble before import \"C\""
    preamble = "\n".join(ln for ln in m.group(1).splitlines() if not ln.strip().startswith("#cgo"))
    names = sorted({n for _, n, _, _ in go_calls()})
    c = tmp_path / "cgo_preamble.c"
    c.write_text(preamble + "\n#include <stdio.h>\nint main(void) {\n"
                 + "".join(f"    printf(\"%p\\n\", (void*)&{n});\n" for n in names) + "    return 0;\n}\n")
    exe = tmp_path / "cgo_preamble"
    libdir = os.path.dirname(LIB)
    # The same flags as the package's #cgo lines: -I include, -L lib -ldpf_hip, rpath.
    subprocess.run([gcc, "-std=c99", "-Wall", "-Werror", "-I", os.path.join(ROOT, "include"), str(c), "-o", str(exe),
                    "-L", libdir, "-ldpf_hip", f"-Wl,-rpath,{libdir}", "-Wl,--unresolved-symbols=ignore-in-shared-libs"],
                   check=True, capture_output=True, text=True)
    assert exe.exists()
