"""bench.py's host-side helpers for the N > 1 line, without a GPU: the
amd-smi xGMI counter parsing (the one-GPU box's real output, and a
synthetic two-link node), counter deltas against the algorithmic bytes,
and TEMPI_CACHE_DIR resolution (the same rule as tempi_amd/csrc/core/env.cpp)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

# `amd-smi xgmi -m --json` on this pool's one-GPU MI355X box (ROCm 7.2.0)
ONE_GPU = {"xgmi_metric": [[{"gpu": 0, "bdf": "0000:72:00.0", "link_metrics": {
    "bit_rate": {"value": 38, "unit": "Gb/s"}, "max_bandwidth": {"value": 608, "unit": "Gb/s"}, "link_type": "N/A",
    "links": [{"gpu": 0, "bdf": "0000:72:00.0", "read": "N/A", "write": "N/A"}]}}]]}


def node(read_kb, write_kb):
    """two GPUs, one link each way, with accumulated data counters in KB"""
    gpus = []
    for g in (0, 1):
        gpus.append({"gpu": g, "link_metrics": {"links": [
            {"gpu": 1 - g, "read": {"value": read_kb[g], "unit": "KB"}, "write": {"value": write_kb[g], "unit": "KB"}},
            {"gpu": g, "read": "N/A", "write": "N/A"}]}})
    return {"xgmi_metric": [gpus]}


def fake_smi(monkeypatch, doc):
    monkeypatch.setattr("shutil.which", lambda name: "/usr/bin/amd-smi")

    def run(cmd, **kw):
        assert cmd[:3] == ["amd-smi", "xgmi", "-m"]
        return subprocess.CompletedProcess(cmd, 0, json.dumps(doc), "")

    monkeypatch.setattr(bench.subprocess, "run", run)


def test_one_gpu_box_has_no_xgmi_counters(monkeypatch):
    fake_smi(monkeypatch, ONE_GPU)
    assert bench.xgmi_snapshot() is None
    d = bench.xgmi_delta(None, None, 11, 1000, 1.0)
    assert d["available"] is False and "SELF" in d["note"]


def test_xgmi_delta_per_iteration(monkeypatch):
    fake_smi(monkeypatch, node([100, 200], [300, 400]))
    a = bench.xgmi_snapshot()
    assert a == {(0, 1): (100 * 1024.0, 300 * 1024.0), (1, 0): (200 * 1024.0, 400 * 1024.0)}
    fake_smi(monkeypatch, node([100 + 1100, 200 + 1100], [300 + 1100, 400 + 1100]))
    b = bench.xgmi_snapshot()
    d = bench.xgmi_delta(a, b, 11, 2 * 100 * 1024, 0.5)
    assert d["available"] and d["read_bytes"] == d["write_bytes"] == 2 * 1100 * 1024
    assert d["per_unit_bytes"] == 2 * 100 * 1024 and d["algorithmic_per_unit_bytes"] == 2 * 100 * 1024
    assert d["counter_GBps"] == round(2 * 1100 * 1024 / 0.5 / 1e9, 1) and d["links_reporting"] == 2


def test_smi_units():
    assert bench._smi_bytes({"value": 3, "unit": "KB"}) == 3072
    assert bench._smi_bytes({"value": 2, "unit": "MB"}) == 2 << 20
    assert bench._smi_bytes("N/A") is None
    assert bench._smi_bytes(5) == 5.0


@pytest.mark.parametrize("env,expect", [({"TEMPI_CACHE_DIR": "/x/c"}, "/x/c"),
                                        ({"XDG_CACHE_HOME": "/x/xdg"}, "/x/xdg/tempi"),
                                        ({"HOME": "/x/h"}, "/x/h/.tempi")])
def test_cache_dir(monkeypatch, env, expect):
    for k in ("TEMPI_CACHE_DIR", "XDG_CACHE_HOME", "HOME"):
        monkeypatch.delenv(k, raising=False)
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    assert bench.tempi_cache_dir() == expect


def test_section_error_is_recorded():
    sec = bench.Sections({"metric": "m"}, 0, 60.0)
    try:
        r = sec.run("halo", lambda: (_ for _ in ()).throw(RuntimeError("halo exchange failed rc=3")))
    finally:
        sec.done()
    assert r == {"error": "RuntimeError: halo exchange failed rc=3"}


def test_section_deadline_prints_the_line_so_far():
    code = ("import sys, time; sys.path.insert(0, %r); import bench\n"
            "rec = {'metric': 'm', 'value': 1.0, 'unit': 'GB/s', 'n_gpus': 1}\n"
            "sec = bench.Sections(rec, 0, 0.5)\n"
            "sec.run('halo', time.sleep, 30)\n") % ROOT
    r = subprocess.run([sys.executable, "-c", code], stdout=subprocess.PIPE, text=True, timeout=60)
    line = json.loads(r.stdout.strip().splitlines()[-1])
    assert r.returncode == 0 and line["value"] == 1.0
    assert line["incomplete"] == {"section": "halo", "deadline_s": 0.5}


def _brute_classes(bl, st, n, first):
    """line classes of n rows, byte by byte (small cases only)"""
    lines = {}
    for r in range(n):
        for b in range(first + r * st, first + r * st + bl):
            lines.setdefault(b // 128, [0, 0])[(b % 128) // 64] += 1
    touched = len(lines)
    partial = sum(any(0 < s < 64 for s in v) for v in lines.values())
    whole = sum(v == [64, 64] for v in lines.values())
    return touched, partial, whole, touched - partial - whole


@pytest.mark.parametrize("bl,st,n,first", [(512, 1024, 64, 0), (8, 16, 4096, 0), (128, 144, 256, 0),
                                           (64, 512, 128, 0), (3, 19, 2000, 38), (24, 4608, 40, 24),
                                           (1, 2, 9000, 5), (2048, 2064, 40, 0)])
def test_touched_line_classes_exact(bl, st, n, first):
    """the sampled, period-scaled count equals a byte-by-byte count when the
    sample covers every row"""
    got = bench._line_classes(bl, st, n, first)
    assert tuple(round(x, 6) for x in got) == _brute_classes(bl, st, n, first)


def test_touched_model_headline_and_narrow_rows():
    # headline: 512-B rows at 1024: reads 4 whole lines per row, writes whole lines
    m = bench.touched_model(512, 1024, 1, 1 << 21, 0, 0)
    assert m["pack_bytes"] == m["unpack_bytes"] == 2 * (1 << 30)
    # 8 : 16, 1 GiB: every line read whole (2x the payload), every line has partly written sectors
    m = bench.touched_model(8, 16, 1, 1 << 27, 0, 0)
    lines = (1 << 31) // 128
    assert m["pack_bytes"] == pytest.approx(lines * 128 + (1 << 30))
    assert m["unpack_bytes"] == pytest.approx((1 << 30) + lines * bench.LINE_WRITE_PARTIAL)
    # 64 : 512: one whole sector per touched line, at the calibrated cost of that sparsity
    m = bench.touched_model(64, 512, 1, 1 << 24, 0, 0)
    assert m["unpack_bytes"] == pytest.approx((1 << 30) + (1 << 24) * 125.0)
    # the half-line cost rises with the stride and stays within the calibration
    costs = [bench.half_line_cost(s) for s in (64, 128, 192, 256, 512, 1024, 4096, 65536)]
    assert costs == sorted(costs) and costs[0] == 90.0 and costs[-1] == 140.0


def test_type_commit_cost_section():
    """the line's type_commit section: the reference's bench_type_commit
    shapes through libtempi and through the library alone"""
    r = bench.type_commit_cost()
    for k in ("tempi", "library"):
        assert 0 < r[k]["commit_us_median"] <= r[k]["commit_us_max"]
        assert set(r[k]["per_factory_median_us"]) == {"subarray", "byte_v_hv", "byte_v1_hv_hv", "byte_vn_hv_hv",
                                                      "subarray_v"}


# ---- the driver's line: bounded size, parseable, every section summarised ----

def _full_n1_record():
    """round 2's fully populated N = 1 record (35 KB as printed then), with the
    1 GiB cpu_baseline sample of this round"""
    rec = json.load(open(os.path.join(ROOT, "profiles", "r02", "bench_line_s15.json")))
    rec["halo"]["grid"], rec["halo"]["dims"] = 512, [1, 1, 1]
    return rec


def _n8_record():
    """a synthetic N = 8 record with every N > 1 section at its largest"""
    rec = json.load(open(os.path.join(ROOT, "profiles", "r02", "bench_line_torchrun_n2_s13.json")))
    rec["n_gpus"] = 8
    for name, g in (("halo", 512), ("halo_weak", 1024)):
        rec[name]["grid"], rec[name]["dims"] = g, [2, 2, 2]
        rec[name]["rank0_phase_us"] = {"isend": 1234.5, "irecv": 2345.6, "wait": 34567.8}
        rec[name]["xgmi_counters"] = {"available": True, "per_unit_bytes": 123456789012, "read_bytes": 1 << 40}
    for p in rec["pingpong_1d"]["points"]:
        p["pairs"] = 4
    for name in ("alltoallv", "nbr_alltoallv"):
        for p in rec[name]["points"]:
            p["ranks"] = 8
    rec["perf_model"]["auto_model"] = "/some/very/long/path/" + "x" * 200 + "/perf.json"
    # the transport block (round 6), every route used, with the largest counts
    big = {"messages": 123456789, "bytes": 123456789012345}
    rec["transport"] = {"over": "every N > 1 section, all ranks",
                        "routes": {k: dict(big) for k in ("ipc", "ipc_copy", "oneshot", "staged", "device", "direct")},
                        "library_sends": 123456789, "self_matched": 123456, "batches": 1234567, "ticket_batches": 12345,
                        "canary_ok": 56, "canary_fail": 0, "ipc_threshold": {"block_24": 4096, "block_512": 4096,
                                                                              "from_node_perf_json": True},
                        "perf_json_measured_on_node": True}
    return rec


def test_transport_block_in_the_line():
    """the N > 1 line carries the transport block's
    per-route [messages, bytes], library sends, canaries, the IPC threshold
    and where the model came from; with the ranks on one GPU the canaries
    are null with the reason"""
    rec = _n8_record()
    t = bench.compact_line(rec, False)["transport"]
    assert t["routes"]["ipc"] == [123456789, 123456789012345] and t["canary_ok"] == 56
    assert t["ipc_threshold"]["from_node_perf_json"] is True and t["perf_json_measured_on_node"] is True
    rec["transport"].update(canary_ok=None, canary_fail=None, canary_note="shared GPU: ...")
    t = bench.compact_line(rec, True)["transport"]
    assert t["canary_ok"] is None and t["null_because"] == "shared GPU"


@pytest.mark.parametrize("which", ["n1", "n8", "n8_shared"])
def test_line_is_bounded_and_parses(which):
    rec = _full_n1_record() if which == "n1" else _n8_record()
    shared = which == "n8_shared"
    if shared:
        bench.null_shared_gpu_fractions(rec)
    line = bench.compact_line(rec, shared, "gpurun_out/bench_detail_n8.json")
    s = json.dumps(line)
    assert len(s) < 4096 and len(s) <= bench.LINE_LIMIT
    back = json.loads(s)
    # the contract's keys, the headline's roofline and cpu_baseline survive whole
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config"):
        assert back[k] == rec[k]
    for k in ("bound", "achieved", "peak", "unit", "frac", "traffic"):
        assert back["roofline"][k] == rec["roofline"][k]
    assert "dropped" not in back  # nothing had to be dropped to fit
    if which == "n1":
        assert back["cpu_baseline"]["value"] == rec["cpu_baseline"]["value"]
        assert back["cpu_baseline"]["cores"] == 1 and back["cpu_baseline"]["kind"] == "reference"
        assert back["sweep"]["points"] == 64 and len(back["sweep"]["worst_touched"]) == 3
        assert back["halo"]["us_per_iter"] == rec["halo"]["us_per_iter"] and back["halo"]["bound"] == "hbm"
        assert back["mpi_pack"]["errors"] == 0 and back["config1"]["speedup"] == rec["config1"]["speedup"]
    else:
        for name in ("halo", "halo_weak", "pingpong", "pingpong_1d", "alltoallv", "nbr_alltoallv", "perf_model"):
            assert name in back, name
        assert len(back["alltoallv"]["points"]) == 3 and back["halo"]["dims"] == [2, 2, 2]
    if shared:
        assert back["shared_gpu"] is True and back["halo"]["frac"] is None and back["halo"]["aggregate_frac"] is None
        assert all(p[-1] is None for n in ("pingpong", "pingpong_1d", "alltoallv", "nbr_alltoallv")
                   for p in back[n]["points"])


def test_line_overflow_drops_sections_in_order():
    rec = _full_n1_record()
    rec["mpi_pack"]["pack_speedup_geomean_by_target"] = {str(i): 1.0 for i in range(400)}
    line = bench.compact_line(rec, False, None)
    assert len(json.dumps(line)) <= bench.LINE_LIMIT
    assert line["dropped"][0] == "mpi_pack" and "roofline" in line and "cpu_baseline" in line


def test_line_section_errors_are_short():
    rec = _full_n1_record()
    rec["halo"] = {"error": "RuntimeError: " + "x" * 5000}
    line = bench.compact_line(rec, False, None)
    assert len(line["halo"]["error"]) <= 160 and len(json.dumps(line)) <= bench.LINE_LIMIT


def test_shared_gpu_fractions_are_null():
    rec = _n8_record()
    bench.null_shared_gpu_fractions(rec)
    r = rec["halo"]["roofline"]
    assert r["frac"] is None and r["aggregate_frac"] is None and "note" in r
    assert all(q["xgmi_frac"] is None for q in rec["pingpong_1d"]["points"])


def test_sweep_traffic_keeps_stdout_to_the_bench_line(monkeypatch, capsys):
    """bench.py's stdout carries exactly one JSON line (the driver's
    contract): the sweep counter check (tools/sweep_pmc.py) records its shapes
    in the bench detail, never on stdout. Profiler and timing children are
    replaced here by fixed numbers."""
    import shutil

    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import sweep_pmc

    monkeypatch.setattr(shutil, "which", lambda name: "/usr/bin/" + name)
    for k in [k for k in os.environ if k.startswith("ROCPROF")]:
        monkeypatch.delenv(k)
    monkeypatch.setenv("LD_PRELOAD", "")
    info = {"planes": [1, 1000, 0, 0], "shape": "2d rows=1000 stride=40", "payload": 24000,
            "pack_ms": 0.01, "unpack_ms": 0.02}
    monkeypatch.setattr(sweep_pmc, "profile", lambda spec, counter, outdir: (info, {"pack": 20000.0, "unpack": 12000.0}))
    monkeypatch.setattr(sweep_pmc, "timed", lambda spec: info)
    recs = bench.sweep_traffic(["2:24:40"])
    assert recs and recs[0]["spec"] == "2:24:40" and "pack_model_over_counted" in recs[0]
    assert capsys.readouterr().out == ""
    sweep_pmc.run(["2:24:40"], None)  # (the command line still prints its records)
    assert json.loads(capsys.readouterr().out)["spec"] == "2:24:40"
