"""Compare campaign: run/run_compare.sh -> ftrun -> drivers ->
analysis/check_compare.py -> data_compare CSVs (the reference's slurm/test_compare.slurm +
analysis/check_compare.py layout)."""
import csv
import importlib.util
import json
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "fault-tolerant_amd")
RUN = os.path.join(PKG, "run")


def _checker(out, data):
    os.environ["FTAR_CMP_OUT"], os.environ["FTAR_CMP_DATA"] = str(out), str(data)
    try:
        spec = importlib.util.spec_from_file_location("check_compare", os.path.join(PKG, "analysis", "check_compare.py"))
        m = importlib.util.module_from_spec(spec)
        spec.loader.exec_module(m)
    finally:
        del os.environ["FTAR_CMP_OUT"], os.environ["FTAR_CMP_DATA"]
    return m


def _stdout(np_, size, t, results, header_on_all=False):
    lines = []
    for r, v in enumerate(results):
        if header_on_all or r == 0:
            lines += [f"P: {np_}", f"Size: {size}", f"Time: {t:f}"]
        lines.append(f"Hello from {r} of {np_} and the result is: {v}")
    return "\n".join(lines) + "\n"


def _rows(path):
    return list(csv.DictReader(open(path), delimiter=";"))


def test_check_compare_rows_and_errors(tmp_path):
    out, data = tmp_path / "out", tmp_path / "data"
    out.mkdir()
    m = _checker(out, data)
    good = ((4 * 3 // 2) % 17) * 1000
    (out / "rd.txt").write_text(_stdout(4, 1000, 0.25, [good] * 4, header_on_all=True))
    (out / "original_rd.txt").write_text(_stdout(4, 1000, 0.125, [good] * 4))
    (out / "raben.txt").write_text(_stdout(4, 1000, 0.5, [good] * 3 + [good + 1], header_on_all=True))
    (out / "original_raben.txt").write_text(_stdout(4, 1000, 0.1, [good] * 4))
    assert m.main() == 1
    assert _rows(data / "rd.csv") == [{"NP": "4", "SIZE": "1000", "TIME": "0.25", "RESULT": str(good)}]
    assert _rows(data / "original_rd.csv")[0]["TIME"] == "0.125"
    assert not (data / "raben.csv").exists() and not (data / "original_raben.csv").exists()
    err = (out / "error.txt").read_text()
    assert err.startswith("RABEN: [4, 1000, 0.5,") and "RABEN_O: [4, 1000, 0.1," in err
    # a missing rank (fewer Hello lines than P) is an error as in the reference
    (out / "raben.txt").write_text(_stdout(4, 1000, 0.5, [good] * 3, header_on_all=True))
    assert m.check_pair("raben", "original_raben", "RABEN") is False
    (out / "raben.txt").write_text(_stdout(4, 1000, 0.5, [good] * 4, header_on_all=True))
    assert m.check_pair("raben", "original_raben", "RABEN") is True
    assert len(_rows(data / "raben.csv")) == 1 and len(_rows(data / "rd.csv")) == 1


def test_run_compare_campaign_hostsim(hostsim, tmp_path):
    """The campaign loop end to end on CPU: host-sim FT drivers in all four slots (the
    vendor baseline needs RCCL on a GPU; it runs in the GPU test below)."""
    hs = os.path.join(ROOT, "tests", "hostsim", "_build", "src")
    env = dict(os.environ, FTAR_CMP_NPS="3 4", FTAR_CMP_BUF_MIN="1", FTAR_CMP_BUF_MAX="64",
               FTAR_CMP_RD=f"{hs}/rd/main", FTAR_CMP_RABEN=f"{hs}/raben/main",
               FTAR_CMP_ORIG_RD=f"{hs}/rd/main", FTAR_CMP_ORIG_RABEN=f"{hs}/raben/main",
               FTAR_CMP_OUT=str(tmp_path / "out"), FTAR_CMP_DATA=str(tmp_path / "data"),
               FTAR_HOSTSIM_TAG="compare", FTAR_FILL_OFFSET="3")
    os.makedirs(tmp_path / "out")
    cp = subprocess.run(["./run_compare.sh", "1"], cwd=RUN, env=env, capture_output=True, text=True, timeout=300)
    subprocess.run("rm -f /dev/shm/ftarhs-compare-*", shell=True)
    assert cp.returncode == 0, cp.stdout[-2000:] + cp.stderr[-2000:]
    for name in ("rd", "original_rd", "raben", "original_raben"):
        rows = _rows(tmp_path / "data" / f"{name}.csv")
        assert len(rows) == 2 * 7, (name, rows)
        for r in rows:  # buffer[i] = rank + 3 (FTAR_FILL_OFFSET): the closed form with the offset
            n, size = int(r["NP"]), int(r["SIZE"])
            assert int(r["RESULT"]) == ((n * (n - 1) // 2 + 3 * n) % 17) * size
    assert not (tmp_path / "out" / "error.txt").exists()


@pytest.mark.gpu
def test_run_compare_campaign_gpu(tmp_path):
    """All four executables on the GPU (NP = 1: the box has one GPU and RCCL refuses two
    ranks on one device), including the RCCL vendor baseline.  The inputs are rank + 5
    (FTAR_FILL_OFFSET), so every RESULT is the nonzero closed form 5 * SIZE, not the 0 a
    one-rank run of the reference's input gives whatever the drivers compute.  Two sizes: one
    int and 2^20 ints (4 MiB, past every small-call path) -- ADVICE r05."""
    env = dict(os.environ, FTAR_CMP_NPS="1", FTAR_CMP_BUF_MIN="1", FTAR_CMP_BUF_MAX=str(1 << 20),
               FTAR_CMP_BUF_MUL=str(1 << 20),
               FTAR_CMP_OUT=str(tmp_path / "out"), FTAR_CMP_DATA=str(tmp_path / "data"), FTAR_FILL_OFFSET="5")
    os.makedirs(tmp_path / "out")
    cp = subprocess.run(["./run_compare.sh", "1"], cwd=RUN, env=env, capture_output=True, text=True, timeout=600)
    assert cp.returncode == 0, cp.stdout[-2000:] + cp.stderr[-2000:]
    for name in ("rd", "original_rd", "raben", "original_raben"):
        rows = _rows(tmp_path / "data" / f"{name}.csv")
        assert sorted(int(r["SIZE"]) for r in rows) == [1, 1 << 20], (name, rows, cp.stdout[-2000:])
        assert all(int(r["RESULT"]) == 5 * int(r["SIZE"]) and int(r["SIZE"]) > 0 for r in rows), rows


def _analyze():
    spec = importlib.util.spec_from_file_location("ftar_analyze", os.path.join(PKG, "analysis", "analyze.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def test_analyze_compare_and_fault_tables(tmp_path):
    a = _analyze()
    ft, orig = tmp_path / "rd.csv", tmp_path / "original_rd.csv"
    ft.write_text("NP;SIZE;TIME;RESULT\n4;16;0.2;96\n4;16;0.4;96\n4;32;0.5;192\n8;16;1.0;208\n")
    orig.write_text("NP;SIZE;TIME;RESULT\n4;16;0.1;96\n4;32;0.25;192\n8;16;0.5;208\n8;64;1;0\n")
    m = a.compare_table(str(ft), str(orig), "RD")
    assert list(m["NP"]) == [4, 4, 8] and list(m["SIZE"]) == [16, 32, 16]
    assert list(m["TIME_RD"].round(6)) == [0.3, 0.5, 1.0]
    assert list(m["RATIO_RD"].round(6)) == [3.0, 2.0, 2.0]
    log = tmp_path / "log.csv"
    log.write_text("N;DELAY;BUF SIZE;KILLED;TIME;DEADLOCK;SEGFAULT;ABORT;RIGHT RESULT\n"
                   "5;2;100;0;1.0;False;False;False;True\n5;2;100;0;3.0;False;False;False;True\n"
                   "5;3;100;1;2.0;False;False;False;True\n5;3;100;1;31.0;True;False;False;False\n")
    t = a.fault_table(str(log))
    assert t.to_dict("records")[0]["count"] == 2 and t.to_dict("records")[0]["mean"] == 2.0
    assert t.to_dict("records")[1]["count"] == 1 and t.to_dict("records")[1]["max"] == 2.0


def test_analyze_clean_sampling(tmp_path):
    a = _analyze()
    src = tmp_path / "log.csv"
    rows = ["N;KILLED;TIME"] + [f"{n};{k};{i}" for n in (5, 9) for k in (0, 1, 5) for i in range(80)]
    src.write_text("\n".join(rows) + "\n")
    kept = a.clean(str(src), str(tmp_path / "out.csv"), [5, 9])
    assert kept == 4 * 50
    out = _rows(tmp_path / "out.csv")
    assert {(r["N"], r["KILLED"]) for r in out} == {("5", "0"), ("5", "1"), ("9", "0"), ("9", "1")}
    # deterministic (seed 42 before every class pair, as clean_data.py)
    a.clean(str(src), str(tmp_path / "out2.csv"), [5, 9])
    assert (tmp_path / "out.csv").read_text() == (tmp_path / "out2.csv").read_text()


def test_analyze_figures(tmp_path):
    """Every figure of the reference's analysis scripts is produced (matplotlib, Agg):
    compare panels + ratio, the 0-vs-1-killed boxplot, the outcome pie, and bench.py's
    size sweep (FT vs RCCL)."""
    a = _analyze()
    ft, orig = tmp_path / "rd.csv", tmp_path / "original_rd.csv"
    ft.write_text("NP;SIZE;TIME;RESULT\n" + "".join(f"{n};{s};{s * 1e-6 * n};0\n" for n in (4, 8) for s in (1, 64, 4096)))
    orig.write_text("NP;SIZE;TIME;RESULT\n" + "".join(f"{n};{s};{s * 5e-7 * n};0\n" for n in (4, 8) for s in (1, 64, 4096)))
    a.plot_compare(a.compare_table(str(ft), str(orig), "RD"), "RD", str(tmp_path / "cmp.png"))
    log = tmp_path / "log.csv"
    log.write_text("N;DELAY;BUF SIZE;KILLED;TIME;DEADLOCK;SEGFAULT;ABORT;RIGHT RESULT\n" +
                   "".join(f"{n};2;100;{k};{1 + k + i / 10};False;False;{'True' if k and i == 0 else 'False'};True\n"
                           for n in (5, 9) for k in (0, 1) for i in range(5)))
    a.plot_fault(a.fault_frame(str(log)), "Rabenseifner", str(tmp_path / "fault.png"))
    cnt = a.outcome_counts(str(log))
    assert cnt == {"recovered": 8, "abort_after_recovery": 2, "abort": 0, "wrong_result": 0, "deadlock": 0}
    a.plot_outcomes(cnt, str(tmp_path / "pie.png"))
    bj = tmp_path / "bench.json"
    bj.write_text(json.dumps({"n_gpus": 8, "size_sweep_us": {
        str(b): {"bytes": b, "raben_us": 50 + b / 1e4, "rd_us": 60 + b / 1e4, "rccl_us": 30 + b / 2e4,
                 "raben_over_rccl": (50 + b / 1e4) / (30 + b / 2e4)} for b in (4, 1024, 1 << 20, 1 << 28)}}) + "\n")
    a.plot_sweep(a.sweep_table(str(bj)), str(tmp_path / "sweep.png"))
    for f in ("cmp.png", "fault.png", "pie.png", "sweep.png"):
        assert (tmp_path / f).stat().st_size > 5000, f


def test_analyze_decisions_from_a_node_line(tmp_path):
    """`analyze.py decisions`: what a node's N > 1 line decides -- the mesh
    form picked, the mid-size gate limit (the largest size up to which every gated column
    beats its ungated twin), the cross-GPU elided-copy verdict, the north-star fractions."""
    a = _analyze()
    mb = 1 << 20
    line = {"n_gpus": 8, "value": 2100.0, "transport": "mesh-u4",
            "transport_selection": {"mesh_ms": 1.02, "mesh_u4_ms": 0.98, "mesh_push_ms": 1.2, "chosen": "mesh_u4",
                                    "inexact": ["mesh_push2"], "failed": {"direct": "boom"}},
            "size_sweep_us": {"small_call_setting": "default (gates, flag-signalled drains)", "gate": 1.0,
                              str(mb): {"bytes": mb, "raben_us": 40, "rd_us": 60},
                              str(2 * mb): {"bytes": 2 * mb, "raben_us": 50, "raben_midgate_us": 45, "rd_us": 70,
                                            "rd_midgate_us": 66},
                              str(8 * mb): {"bytes": 8 * mb, "raben_us": 80, "raben_midgate_us": 70, "rd_us": 120,
                                            "rd_midgate_us": 110},
                              str(16 * mb): {"bytes": 16 * mb, "raben_us": 120, "raben_midgate_us": 125, "rd_us": 200,
                                             "rd_midgate_us": 190}},
            "north_star": {"frac": 0.81, "met": True, "reference_schedule_frac": 0.74, "rehearsal": False},
            "c5_single_kill": {"dead_input_cross_device": "recovered"},
            "exact_on_node": {"all_exact": True},
            "link_calibration": {"single_link_GBps": 64.0}}
    p = tmp_path / "scale8.json"
    p.write_text(json.dumps(dict(line, line="headline")) + "\n" + json.dumps(dict(line, line="final")) + "\n")
    d = a.decisions(a._last_line(str(p)))
    assert d["transport_chosen"] == "mesh_u4" and d["never_fastest"] == ["mesh", "mesh_push"]
    assert d["transport_inexact_or_failed"] == ["direct", "mesh_push2"]
    assert d["gate_max_bytes"] == 8 * mb and d["gate_max_changes"]
    assert d["elide_step0_copy_across_gpus"] and d["north_star_met"] and d["north_star_frac"] == 0.81
    assert d["small_call_setting"].startswith("default") and d["link_GBps"] == 64.0
    # a gated column that loses at the first mid size keeps the library's 1 MiB
    line["size_sweep_us"][str(2 * mb)]["rd_midgate_us"] = 71
    assert a.decisions(line)["gate_max_bytes"] == mb
