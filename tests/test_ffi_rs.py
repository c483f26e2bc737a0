"""CPU check of the Rust FFI source against the C ABI it binds.

There is no rustc in the image, so `adapters/hip_ffi.rs` (the drop-in for rust_lib/src/metal_ffi.rs, whose own
extern block is metal_ffi.rs:10-30) cannot be compiled here.  Instead its `extern "C"` block is parsed and every
declaration is held to the prototype in include/hip_diskann_bridge.h: same function name, same arity, same argument
names in the same order, and each argument / return type equal under the Rust <-> C type map below.  A drifted
argument order (e.g. `nq` vs `ids` in `_ids`) fails here instead of at the extension's link.
"""
from __future__ import annotations

import re
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
RS = ROOT / "duckdb-annsearch_amd" / "adapters" / "hip_ffi.rs"
HDR = ROOT / "include" / "hip_diskann_bridge.h"

# Rust type (whitespace-normalised) -> canonical C type
RUST_TO_C = {
    "i32": "int", "i64": "int64_t", "u32": "uint32_t", "f32": "float", "()": "void",
    "*constf32": "const float*", "*mutf32": "float*",
    "*consti64": "const int64_t*", "*muti64": "int64_t*",
    "*constu32": "const uint32_t*", "*mutu32": "uint32_t*",
    "*constcore::ffi::c_void": "const void*", "*mutcore::ffi::c_void": "void*",
    "*constcore::ffi::c_char": "const char*", "*mutcore::ffi::c_char": "char*",
}
C_ALIASES = {"unsigned int": "uint32_t", "unsigned": "uint32_t"}


def _canon_c(t: str) -> str:
    t = " ".join(t.replace("*", " * ").split())
    const = t.startswith("const ")
    if const:
        t = t[len("const "):]
    ptr = t.count("*")
    base = t.replace("*", "").strip()
    base = C_ALIASES.get(base, base)
    return ("const " if const else "") + base + "*" * ptr


def parse_rust_externs(text: str) -> dict:
    """{name: (ret, [(arg, c_type), ...])} of every fn in the file's `extern "C" { ... }` blocks."""
    out = {}
    for block in re.findall(r'extern\s+"C"\s*\{(.*?)\n\}', text, flags=re.S):
        for m in re.finditer(r"fn\s+(\w+)\s*\((.*?)\)\s*(?:->\s*([^;]+))?;", block, flags=re.S):
            name, args, ret = m.group(1), m.group(2), (m.group(3) or "()").strip()
            params = []
            for a in [x.strip() for x in args.split(",") if x.strip()]:
                an, at = a.split(":", 1)
                key = re.sub(r"\s+", "", at)
                if key not in RUST_TO_C:
                    raise AssertionError(f"{name}: Rust type {at!r} has no entry in the type map")
                params.append((an.strip(), RUST_TO_C[key]))
            rkey = re.sub(r"\s+", "", ret)
            if rkey not in RUST_TO_C:
                raise AssertionError(f"{name}: Rust return type {ret!r} has no entry in the type map")
            out[name] = (RUST_TO_C[rkey], params)
    return out


def parse_c_prototypes(text: str) -> dict:
    """{name: (ret, [(arg, c_type), ...])} of every function prototype in the header."""
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    text = re.sub(r"^\s*#.*$", "", text, flags=re.M)
    out = {}
    for m in re.finditer(r"([A-Za-z_][\w\s\*]*?)\b(\w+)\s*\(([^()]*)\)\s*;", text):
        ret, name, args = m.group(1).strip(), m.group(2), m.group(3).strip()
        params = []
        if args and args != "void":
            for a in [x.strip() for x in args.split(",")]:
                am = re.match(r"(.*?)(\w+)$", a, flags=re.S)
                params.append((am.group(2), _canon_c(am.group(1))))
        out[name] = (_canon_c(ret), params)
    return out


def compare(rs: dict, hdr: dict) -> list:
    """Mismatches between the Rust externs and the header (empty list: identical)."""
    bad = []
    for name, (ret, params) in rs.items():
        if name not in hdr:
            bad.append(f"{name}: not declared in {HDR.name}")
            continue
        cret, cparams = hdr[name]
        if ret != cret:
            bad.append(f"{name}: returns {ret} in Rust, {cret} in C")
        if len(params) != len(cparams):
            bad.append(f"{name}: {len(params)} arguments in Rust, {len(cparams)} in C")
            continue
        for i, ((rn, rt), (cn, ct)) in enumerate(zip(params, cparams)):
            if rn.lower() != cn.lower():
                bad.append(f"{name}: argument {i} is `{rn}` in Rust, `{cn}` in C")
            if rt != ct:
                bad.append(f"{name}: argument {i} (`{rn}`) is {rt} in Rust, {ct} in C")
    return bad


def test_hip_ffi_externs_match_the_c_bridge():
    rs = parse_rust_externs(RS.read_text())
    hdr = parse_c_prototypes(HDR.read_text())
    # the bridge's three reference entry points (metal_ffi.rs:10-30) and every extension call the Rust side uses
    for n in ("diskann_hip_available", "diskann_hip_batch_distances", "diskann_hip_multi_batch_distances",
              "diskann_hip_register_db", "diskann_hip_multi_batch_distances_ids", "diskann_hip_release_db",
              "diskann_hip_register_graph", "diskann_hip_search_batch_resident", "diskann_hip_search_batch"):
        assert n in rs, f"{n} missing from hip_ffi.rs"
    assert compare(rs, hdr) == []


@pytest.mark.parametrize("mutation", ["swap", "type", "arity", "rename"])
def test_hip_ffi_checker_catches_drift(mutation):
    """Negative controls: the checker rejects a swapped argument order, a wrong pointer type, a dropped argument and a
    renamed argument in the Rust block."""
    text = RS.read_text()
    src = "        nq: i32,\n        ids: *const u32,\n"
    assert src in text
    if mutation == "swap":
        text = text.replace(src, "        ids: *const u32,\n        nq: i32,\n", 1)
    elif mutation == "type":
        text = text.replace(src, "        nq: i32,\n        ids: *const i64,\n", 1)
    elif mutation == "arity":
        text = text.replace(src, "        nq: i32,\n", 1)
    else:
        text = text.replace(src, "        nq: i32,\n        labels: *const u32,\n", 1)
    rs = parse_rust_externs(text)
    hdr = parse_c_prototypes(HDR.read_text())
    bad = compare(rs, hdr)
    assert bad and all("diskann_hip_multi_batch_distances_ids" in b for b in bad), bad
