"""The stdout JSON line of bench.py stays small enough for the driver to parse (the 25.8 KB line of round 4
was cut by the driver's stdout tail and left the headline unmeasured). CPU-only: the compactor runs on the full
record bench.py wrote in round 4 (profiles/r04_bench.json, every config's roofline with notes and PMC detail)."""
import json
import os

import bench

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _full():
    with open(os.path.join(ROOT, "profiles", "r04_bench.json")) as f:
        return json.load(f)


def test_compact_line_fits_and_keeps_the_headline():
    full = _full()
    assert len(json.dumps(full)) > 20000  # the record that was not parsed
    s = bench.compact_line(full)
    assert len(s) <= bench.STDOUT_LINE_LIMIT
    assert "\n" not in s
    out = json.loads(s)
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config", "loss"):
        assert out[k] == full[k], k
    r = out["roofline"]
    for k in ("bound", "achieved", "peak", "unit", "frac", "traffic"):
        assert r[k] == full["roofline"][k], k
    assert r["by_pass"]["conv_wgrad"][2] == full["roofline"]["by_pass"]["conv_wgrad"]["TFLOP/s"]
    assert r["hbm_kernels"]["frac"] == full["roofline"]["hbm_kernels"]["frac"]
    assert out["cpu_baseline"]["value"] == full["cpu_baseline"]["value"]
    assert out["cpu_baseline"]["kind"] == "port" and out["cpu_baseline"]["cores"] == full["cpu_baseline"]["cores"]
    assert set(out["configs"]) == set(full["configs"])
    for name, c in full["configs"].items():
        e = out["configs"][name]
        assert e["value"] == c["value"] and e["ms_per_step"] == c["ms_per_step"]
        assert e["frac"] == c["roofline"]["frac"]
        assert e["cpu_baseline"] == (c["cpu_baseline"] or {}).get("value")
    assert out["parity"]["pass"] is True and out["parity"]["max_rel_err"] == full["parity"]["max_rel_err"]


def test_compact_line_drops_the_config_block_before_the_headline():
    full = _full()
    big = dict(full)
    big["configs"] = {f"x{i}": full["configs"]["c5"] for i in range(60)}
    out = json.loads(bench.compact_line(big))
    assert "configs" not in out and out["value"] == full["value"] and out["roofline"]["frac"] == full["roofline"]["frac"]


def test_detail_file_roundtrip(tmp_path):
    full = _full()
    p = bench.write_detail(full, str(tmp_path / "sub" / "detail.json"))
    with open(p) as f:
        assert json.load(f) == full
