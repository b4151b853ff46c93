"""Host-side checks of the measurement tools DESIGN.md §9 and §12 cite:
tools/traffic_ratios.py recomputes every traffic ratio from the committed
profiles, and tools/c5_timeline.py reads a rocprofv3 kernel trace of the C5
step (here a synthetic one)."""
import csv
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_traffic_ratios_from_committed_profiles():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "traffic_ratios.py")], capture_output=True,
                       text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    rows = [l.split() for l in r.stdout.splitlines()[1:] if l.strip()]
    kernels = {(row[0], row[1]): float(row[-1]) for row in rows}
    # the step kernels of every config are there, each moving at least its algorithmic bytes
    assert ("c2", "chachapoly_duplex_solo<true>") in kernels
    assert ("c3", "gcm_duplex_fused<false>") in kernels
    assert any(k[0] == "c5" and k[1].startswith("chachapoly_seg_ragged") for k in kernels)
    for k, ratio in kernels.items():
        assert 0.98 <= ratio < 2.0, (k, ratio)


def test_c5_timeline_on_synthetic_trace(tmp_path):
    d = tmp_path / "trace"
    d.mkdir()
    names = ["void na::gcm_ragged_staged<false, true, 1024, false, 2, 8>(na::RaggedArgs)",
             "na::seg_plan_count(na::RecDesc const*, unsigned int, na::SegPlanHdr*)",
             "void na::chachapoly_seg_ragged<false>(na::RaggedArgs, na::SegPlanHdr*, unsigned int const*)",
             "void na::gcm_ragged_staged<true, true, 1024, false, 2, 8>(na::RaggedArgs)",
             "void na::chachapoly_seg_ragged<true>(na::RaggedArgs, na::SegPlanHdr*, unsigned int const*)"]
    rows = []
    for step in range(3):
        t = step * 2_000_000
        spans = [(0, 760_000), (5_000, 450_000), (450_000, 1_060_000), (760_000, 1_800_000), (1_500_000, 2_000_000)]
        for n, (a, b) in zip(names, spans):
            rows.append({"Kernel_Name": n, "Start_Timestamp": t + a, "End_Timestamp": t + b})
    with open(d / "run_kernel_trace.csv", "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=["Kernel_Name", "Start_Timestamp", "End_Timestamp"])
        w.writeheader()
        w.writerows(rows)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "c5_timeline.py"), str(d), "2"],
                       capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stderr
    last = r.stdout.strip().splitlines()[-1]
    assert "mean span 2000.0 us" in last, r.stdout
    # kernel sum excludes the plan kernels: 760 + 610 + 1040 + 500 = 2910 us
    assert "mean kernel sum 2910.0 us" in last, r.stdout
