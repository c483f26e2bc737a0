"""AddressSanitizer + UndefinedBehaviorSanitizer builds of the CPU-side code (the reference has no
sanitizer build either; VERDICT r05 "What's missing" 4).

* The oracle (`oracle/oracle.c`) with its self-test driver (`oracle/oracle_selftest.c`), built by `make -C oracle
  sanitize` with `-fsanitize=address,undefined -fno-sanitize-recover=all` (leak checking on): every entry point on
  small seeded inputs — Flat (both heap paths), IVF (search, search_preassigned, skipped probes, an empty list),
  batch distances, the SQ8 codec, the lock-step DiskANN BFS (fp32 and SQ8 rows) and k-means.
* The FaissIndex flow harness (`tests/harness`), its host code built with `-Xarch_host -fsanitize=address
  -Xarch_host -fsanitize=undefined` (device code uninstrumented: GPU sanitizers are not available on this pool):
  without a device it must still refuse cleanly; on the GPU box it runs the whole flow.
"""
from __future__ import annotations

import os
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
SAN_ORACLE = ROOT / "oracle" / "build" / "oracle_selftest_san"
SAN_HARNESS = ROOT / "tests" / "harness" / "build" / "faiss_index_harness_san"
SAN_MARKERS = ("ERROR: AddressSanitizer", "ERROR: LeakSanitizer", "runtime error:", "UndefinedBehaviorSanitizer")


def _clean(out: str):
    bad = [m for m in SAN_MARKERS if m in out]
    assert not bad, out[-4000:]


def test_oracle_under_asan_ubsan():
    subprocess.run(["make", "-s", "-C", str(ROOT / "oracle"), "sanitize"], check=True)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0", UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([str(SAN_ORACLE)], capture_output=True, text=True, timeout=300, env=env)
    _clean(r.stdout + r.stderr)
    assert r.returncode == 0 and "all checks passed" in r.stdout, r.stdout + r.stderr


def _build_harness(hipann_mod, oracle):
    subprocess.run(["make", "-s", "-C", str(ROOT / "tests" / "harness"), "sanitize"], check=True)
    assert SAN_HARNESS.exists()


def test_sanitized_harness_refuses_without_gpu(hipann_mod, oracle):
    _build_harness(hipann_mod, oracle)
    if hipann_mod.is_available():
        pytest.skip("a GPU is present: the no-device exit is not observable")
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0")
    r = subprocess.run([str(SAN_HARNESS)], capture_output=True, text=True, timeout=120, env=env)
    _clean(r.stdout + r.stderr)
    assert r.returncode == 2 and "no gfx950 HIP device" in r.stdout


@pytest.mark.gpu
def test_sanitized_harness_flow(gpu, oracle):
    """The whole FaissIndex flow with the host code under ASan + UBSan (leak checking off: the HIP runtime's own
    process-lifetime allocations are not this code's)."""
    _build_harness(gpu, oracle)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:protect_shadow_gap=0", UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([str(SAN_HARNESS)], capture_output=True, text=True, timeout=900, env=env)
    out = ROOT / "gpurun_out"
    out.mkdir(exist_ok=True)
    (out / "faiss_index_harness_san.log").write_text(r.stdout + r.stderr)
    _clean(r.stdout + r.stderr)
    checks = [l for l in r.stdout.splitlines() if l.startswith("CHECK ")]
    failed = [l for l in checks if " FAIL" in l]
    assert r.returncode == 0 and not failed and len(checks) >= 60, "\n".join(failed) or r.stdout[-3000:] + r.stderr[-2000:]
