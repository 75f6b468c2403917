"""CPU: the host-side analysis tools the roofline record is built with
(tools/rocprof_roofline.py, tools/cycle_trace.py) pick the right launches out of a rocprofv3
kernel trace — the bench's own 20 dispatch-packet-timed roofline launches, not the autotune's
flush-preceded timings before them nor the stream-event round after them; the main cycle, not the
variable-coefficient cycle the bench runs afterwards."""
import csv
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FIELDS = ["Kernel_Name", "Start_Timestamp", "End_Timestamp"]
UNI = "void mlamg::k_rowpat_uni<0, false, 2, 1>(unsigned char const*, ...)"
FLUSH = "void at::native::reduce_kernel<512, 1>(...)"


def _write(path, rows):
    with open(path, "w", newline="") as fh:
        w = csv.DictWriter(fh, fieldnames=FIELDS)
        w.writeheader()
        t = 1000
        for name, dur in rows:
            w.writerow({"Kernel_Name": name, "Start_Timestamp": t, "End_Timestamp": t + dur})
            t += dur + 500


def test_rocprof_roofline_picks_the_dispatch_packet_round(tmp_path):
    rows = []
    # autotune: flush-preceded timings of the same kernel (must not be picked)
    for _ in range(20):
        rows += [(FLUSH, 90000), (UNI, 70000)]
    rows += [("void mlamg::k_sorted<0, false, true, false>(...)", 80000)] * 5
    # the bench's roofline: 20 dispatch-packet-timed launches, then 20 between stream events
    for i in range(20):
        rows += [(FLUSH, 90000), (UNI, 44000 + (i % 2) * 100)]
    for _ in range(20):
        rows += [(FLUSH, 90000), (UNI, 48000)]
    # the variable-coefficient line afterwards flushes before other kernels
    for _ in range(5):
        rows += [(FLUSH, 90000), ("void mlamg::k_sell<0, false>(...)", 120000)]
    trace = tmp_path / "trace.csv"
    _write(trace, rows)
    bench = tmp_path / "bench.json"
    bench.write_text(json.dumps({"roofline": {
        "kernel": "fine-level SpMV, y = A x (rowpat kernel, scipy summation order)",
        "avg_launch_us": 44.05, "algorithmic_bytes_per_launch": 166282496, "frac": 0.47}}) + "\n")
    out_csv = tmp_path / "stats.csv"
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "rocprof_roofline.py"),
                        str(trace), str(bench), str(out_csv)], capture_output=True, text=True,
                       check=True)
    assert "window 20" in r.stdout
    assert "rocprof mean 44.05 us" in r.stdout
    row = list(csv.DictReader(open(out_csv)))[0]
    assert int(row["Calls"]) == 20 and abs(float(row["AverageNs"]) - 44050.0) < 1e-6


def test_cycle_trace_keeps_the_main_cycle(tmp_path):
    fin = "mlamg::k_finalize_norm(...)"
    main = [("void mlamg::k_rowpat_uni<1, false, 2, 1>(...)", 50000),
            ("void mlamg::k_sorted<0, false, true, false>(...)", 80000), (fin, 4000)]
    other = [("void mlamg::k_sell<1, false>(...)", 150000), (fin, 4000)]
    rows = [(fin, 4000)] + main * 6 + other * 6
    trace = tmp_path / "trace.csv"
    _write(trace, rows)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "cycle_trace.py"), str(trace),
                        "5", "k_rowpa"], capture_output=True, text=True, check=True)
    last = r.stdout.strip().splitlines()[-1]
    assert last.startswith("cycles 5  kernels 3")
    assert "busy 134.0 us" in last
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "cycle_trace.py"), str(trace),
                        "5"], capture_output=True, text=True, check=True)
    assert r.stdout.strip().splitlines()[-1].startswith("cycles 5  kernels 2")
