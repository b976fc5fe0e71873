"""tools/traffic.py: a full TX/walk profile rewrites its legs and keeps the single-leg
entries (build3, optsc5) only while their kernel unit's source is unchanged; each leg
carries the engine build it was measured on (bench.py checks that build per leg)."""
import csv
import json
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
TOOL = os.path.join(os.path.dirname(HERE), "tools", "traffic.py")

KERNELS = {"build2": "build_kernel", "forward2": "forward_kernel", "opts5": "options_kernel",
           "layers9": "layers_kernel", "fields9": "fields_kernel"}


def build_str(parse="p1", tx="t1", walks="w1", fields="f1"):
    return "rpkt_gpu src=x gfx950; parse=%s tx=%s walks=%s fields=%s" % (parse, tx, walks, fields)


def fake_profile(d, build, kernels, fetch_kib, write_kib):
    os.makedirs(d, exist_ok=True)
    with open(os.path.join(d, "trace_bench.log"), "w") as fh:
        fh.write("noise\n" + json.dumps({"engine_build": build}) + "\n")
    with open(os.path.join(d, "trace_kernel_stats.csv"), "w", newline="") as fh:
        w = csv.DictWriter(fh, ["Name", "Calls"])
        w.writeheader()
        for k in kernels:
            w.writerow({"Name": k, "Calls": 10})
    for name, val in (("fetch", fetch_kib), ("write", write_kib)):
        with open(os.path.join(d, name + "_counter_collection.csv"), "w", newline="") as fh:
            w = csv.DictWriter(fh, ["Kernel_Name", "Counter_Value"])
            w.writeheader()
            for k in kernels:
                for _ in range(10):                     # the first 5 are skipped as warmup
                    w.writerow({"Kernel_Name": k + "(args)", "Counter_Value": val})


def run(*args):
    subprocess.check_call([sys.executable, TOOL] + [str(a) for a in args],
                          stdout=subprocess.DEVNULL)


def test_full_profile_keeps_single_legs_of_unchanged_units(tmp_path):
    out = tmp_path / "traffic_tx.json"
    b1 = build_str()
    fake_profile(tmp_path / "full1", b1, KERNELS.values(), 100.0, 50.0)
    run(tmp_path / "full1", "tx", out)
    fake_profile(tmp_path / "b3", b1, ["build_kernel"], 1000.0, 70.0)
    run(tmp_path / "b3", "tx:build3", out)
    fake_profile(tmp_path / "oc", b1, ["options_kernel"], 400.0, 60.0)
    run(tmp_path / "oc", "tx:optsc5", out)
    t = json.loads(out.read_text())
    assert set(t["legs"]) == set(KERNELS) | {"build3", "optsc5"}
    assert t["legs"]["build3"]["traffic_bytes_per_launch"] == 1000.0 * 1024 * 2 + 70.0 * 1024
    assert all(v["engine_build"] == b1 for v in t["legs"].values())
    assert "kernel_stats_build3" in t and "kernel_stats_optsc5" in t

    # the walks unit changes: a new full profile keeps build3 (tx unchanged), drops optsc5
    b2 = build_str(walks="w2")
    fake_profile(tmp_path / "full2", b2, KERNELS.values(), 200.0, 80.0)
    run(tmp_path / "full2", "tx", out)
    t = json.loads(out.read_text())
    assert set(t["legs"]) == set(KERNELS) | {"build3"}
    assert t["legs"]["build3"]["engine_build"] == b1
    assert t["legs"]["layers9"]["engine_build"] == b2
    assert t["legs"]["layers9"]["traffic_bytes_per_launch"] == 200.0 * 1024 * 2 + 80.0 * 1024
    assert "kernel_stats_build3" in t and "kernel_stats_optsc5" not in t

    # the tx unit changes too: build3 goes
    fake_profile(tmp_path / "full3", build_str(tx="t2", walks="w2"), KERNELS.values(), 1.0, 1.0)
    run(tmp_path / "full3", "tx", out)
    assert set(json.loads(out.read_text())["legs"]) == set(KERNELS)


def test_read_request_sizes(tmp_path):
    """The optional rdreq pass (scripts/profile.sh): the exact read bytes are 32 n32 +
    64 n64 + 128 n128 per launch (warm-up launches skipped), reported beside
    FETCH_SIZE x2 and their ratio, per TX/walk leg."""
    out = tmp_path / "traffic_tx.json"
    d = tmp_path / "full"
    fake_profile(d, build_str(), KERNELS.values(), 100.0, 50.0)
    with open(os.path.join(d, "rdreq_counter_collection.csv"), "w", newline="") as fh:
        w = csv.DictWriter(fh, ["Kernel_Name", "Counter_Name", "Counter_Value"])
        w.writeheader()
        for k in KERNELS.values():
            for _ in range(10):
                for name, v in (("TCC_EA0_RDREQ_32B_sum", 0.0), ("TCC_EA0_RDREQ_64B_sum", 2.0),
                                ("TCC_EA0_RDREQ_128B_sum", 1600.0), ("TCC_EA0_RDREQ_sum", 1602.0)):
                    w.writerow({"Kernel_Name": k + "(args)", "Counter_Name": name,
                                "Counter_Value": v})
    run(d, "tx", out)
    leg = json.loads(out.read_text())["legs"]["layers9"]
    assert leg["read_bytes_by_request_size"] == 2 * 64 + 1600 * 128
    assert abs(leg["fetch_x2_over_by_size"] - 100.0 * 2048 / (2 * 64 + 1600 * 128)) < 1e-12
    assert leg["rdreq"]["TCC_EA0_RDREQ_sum"] == 1602.0
