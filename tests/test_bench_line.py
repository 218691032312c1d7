"""bench.py's stdout line stays driver-parseable: the round-5
line carried every leg's verbose record (22 KB) and the driver did not parse
it.  The line now holds the contract keys, the headline roofline and
cpu_baseline and one compact summary per leg; the verbose record goes to the
detail file.  Checked here on the round-5 full record itself (the largest
`out` the bench has produced) and on the --dry-run skeleton."""
import copy
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402

R05 = os.path.join(ROOT, "profiles", "r05", "bench_r05f.json")
CONTRACT = ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
            "vs_baseline", "dtype", "data", "config")


def _full():
    return json.load(open(R05))


def test_round5_record_compacts_under_limit():
    out = _full()
    assert len(json.dumps(out)) > 20000  # the line the driver did not parse
    s = bench.compact_line(out, "profiles/bench_detail_last.json")
    assert len(s) < bench.LINE_LIMIT
    line = json.loads(s)
    for k in CONTRACT:
        assert k in line
    assert line["value"] == out["value"]
    assert line["config"]["workload"] == "pallas_msm_2^20_per_gpu"
    r = line["roofline"]
    for k in ("bound", "achieved", "peak", "unit", "frac", "traffic"):
        assert k in r
    assert r["frac"] == out["roofline"]["frac"]
    c = line["cpu_baseline"]
    for k in ("value", "unit", "cores", "kind", "sample"):
        assert k in c
    legs = line["legs"]
    assert legs["accumulator"]["value"] == out["accumulator"]["value"]
    assert legs["accumulator"]["cpu"]["value"] == out["accumulator"]["cpu_baseline"]["value"]
    assert legs["logn22"]["matches"] is True
    assert legs["small_n"]["gpu_us_fresh_bases"]
    assert "kernels_ms" not in s and "per_proof_work" not in s


def test_growth_never_breaks_the_line():
    """Even a record with many more legs stays under the limit (fields, then
    the legs, are dropped; the contract keys never are)."""
    out = _full()
    leg = out["accumulator"]
    for i in range(200):
        out[f"extra_leg_{i}"] = copy.deepcopy(leg)
    s = bench.compact_line(out)
    assert len(s) < bench.LINE_LIMIT
    line = json.loads(s)
    for k in CONTRACT + ("roofline", "cpu_baseline"):
        assert k in line


def test_emit_writes_detail(tmp_path, capsys):
    out = _full()
    p = tmp_path / "d" / "detail.json"
    bench.emit(out, str(p))
    last = capsys.readouterr().out.strip().splitlines()[-1]
    assert len(last) < bench.LINE_LIMIT
    assert json.loads(last)["detail"] == str(p)
    assert json.load(open(p)) == out


def test_dry_run_line():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--dry-run", "--steps", "3"],
                       capture_output=True, text=True, timeout=300, cwd=ROOT)
    assert r.returncode == 0, r.stderr
    last = r.stdout.strip().splitlines()[-1]
    assert len(last) < bench.LINE_LIMIT
    line = json.loads(last)
    for k in CONTRACT:
        assert k in line


def test_final_record_host_scalar_legs():
    """The final round-6 record (the split scalar copy): the host-scalar legs'
    summaries carry the one-copy comparison, and the whole line compacts
    under the limit with every leg matching."""
    out = json.load(open(os.path.join(ROOT, "profiles", "r06", "bench_r06_final3_detail.json")))
    line = json.loads(bench.compact_line(out))
    legs = line["legs"]
    for k in ("host_scalars", "dropin_pm_msm"):
        assert legs[k]["one_copy_ms"] > legs[k]["ms"] > 0, k
        assert legs[k]["matches"] is True, k
    assert all(v.get("matches", True) for v in legs.values())
