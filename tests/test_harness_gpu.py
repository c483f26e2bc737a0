"""The extension's FaissIndex flow over the C ABI — SURVEY §8f ranks 1 and 2, run as a compiled program.

tests/harness/faiss_index_harness.cpp restates FaissIndex::Search / EnsureGpuIndex / Append / Delete / Vacuum
(src/faiss_index.cpp:108-153, :430-500, :708-762, :840-899) with the batched SearchBatch (rank 1, INTEGRATION.md
§1.1) and the append-on-GPU-copy + lazy re-upload changes (rank 2, §1.2), on top of include/hip_ann.h.  The CPU
FAISS index of the restatement is the oracle (test infrastructure).  Each scenario drives a GPU-mode index and
its CPU-mode twin through build → SearchBatch / Search → delete → append → vacuum → lazy re-upload and checks
that SearchBatch(nq) equals the loop of Search(1), that every result equals the CPU path's, that tombstones
are skipped, that appends land on the GPU copy without a re-upload, and that VACUUM's invalidation is followed
by exactly one re-upload.
"""
from __future__ import annotations

import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
HARNESS = ROOT / "tests" / "harness" / "build" / "faiss_index_harness"


def _build(hipann_mod, oracle):
    subprocess.run(["make", "-s", "-C", str(ROOT / "tests" / "harness")], check=True)
    assert HARNESS.exists()


def test_harness_links_and_refuses_without_gpu(hipann_mod, oracle):
    """The program builds against libhipann.so + the oracle and, with no device, fails loudly (exit 2)."""
    _build(hipann_mod, oracle)
    if hipann_mod.is_available():
        pytest.skip("a GPU is present: the no-device exit is not observable")
    r = subprocess.run([str(HARNESS)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 2 and "no gfx950 HIP device" in r.stdout


@pytest.mark.gpu
def test_faiss_index_flow_harness(gpu, oracle):
    _build(gpu, oracle)
    r = subprocess.run([str(HARNESS)], capture_output=True, text=True, timeout=600)
    out = ROOT / "gpurun_out"
    out.mkdir(exist_ok=True)
    (out / "faiss_index_harness.log").write_text(r.stdout + r.stderr)
    checks = [l for l in r.stdout.splitlines() if l.startswith("CHECK ")]
    failed = [l for l in checks if " FAIL" in l]
    assert r.returncode == 0 and not failed and len(checks) >= 60, "\n".join(failed) or r.stdout[-3000:] + r.stderr[-2000:]
