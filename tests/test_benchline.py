"""The bench line the driver parses (bench.py compact_line): bounded size, the contract's headline fields.

r03's line carried every sweep and reached 23.4 KB; the driver returned it unparsed.  These tests rebuild
the line from the full r03 record (profiles/r03/bench_default_final.json, the same shape bench.py now
writes to its detail file) and from a synthetic worst case, and hold it under the budget."""
import copy
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

import bench  # noqa: E402

R03 = ROOT / "profiles" / "r03" / "bench_default_final.json"
HEADLINE = ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
            "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline", "recall_at_10")


def _full():
    return json.loads(R03.read_text().strip().splitlines()[-1])


def test_compact_line_from_r03_record_fits_and_keeps_headline():
    full = _full()
    assert len(json.dumps(full)) > 20000  # the record that did not parse
    line = bench.compact_line(full)
    s = json.dumps(line)
    assert len(s) < bench.LINE_BUDGET < 12000
    for k in HEADLINE:
        assert k in line, k
    assert line["value"] == full["value"]
    for k in ("bound", "achieved", "peak", "unit", "frac", "traffic", "kernel_ms", "frac_vs_survey_bytes"):
        assert k in line["roofline"], k
    for k in ("value", "unit", "cores", "kind"):
        assert k in line["cpu_baseline"], k
    cfg = line["configs"]
    assert cfg["C2_flat_l2_1m_768"]["value"] == full["configs"]["C2_flat_l2_1m_768"]["value"]
    assert cfg["C5_flat_ip_100m_768_sharded"]["frac"] == full["configs"]["C5_flat_ip_100m_768_sharded"]["roofline"]["frac"]
    assert cfg["C4_diskann_1m_1536_sq8"]["kernel_ms"] > 0
    json.loads(s)  # one parseable line


def test_compact_line_worst_case_stays_under_budget():
    """Twice as many configs, with long error strings: the fallback trims to the core fields."""
    full = _full()
    big = copy.deepcopy(full)
    for name, c in list(full["configs"].items()):
        c2 = copy.deepcopy(c)
        c2["error"] = "x" * 5000
        big["configs"][name + "_copy"] = c2
    s = json.dumps(bench.compact_line(big))
    assert len(s) < 12000


def test_emit_writes_detail_and_prints_one_line(tmp_path, capsys, monkeypatch):
    monkeypatch.setattr(bench, "DETAIL_PATH", tmp_path / "detail.json")
    full = _full()
    bench.emit(full, 0)
    out = capsys.readouterr().out.strip().splitlines()
    assert len(out) == 1
    assert json.loads(out[0])["value"] == full["value"]
    assert json.loads((tmp_path / "detail.json").read_text())["configs"].keys() == full["configs"].keys()
    bench.emit(full, 1)  # other ranks print nothing
    assert capsys.readouterr().out == ""
