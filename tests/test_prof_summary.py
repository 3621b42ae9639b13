"""tools/prof_summary.py's HBM accounting (round 5) on a synthetic rocprofv3 counter CSV: only the
counted (last) step's dispatches count, a dispatch whose SQ_WAVES exceeds its grid's waves (a context save and restore:
the save writes every resident wave's registers and the CUs' LDS) is listed under `context_saves` and left out of
`hbm_bytes_per_candidate`, and the run total over the clean dispatches then equals the median dispatch."""
import csv
import json
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
COLS = ["Correlation_Id", "Dispatch_Id", "Agent_Id", "Queue_Id", "Process_Id", "Thread_Id", "Grid_Size", "Kernel_Id",
        "Kernel_Name", "Workgroup_Size", "LDS_Block_Size", "Scratch_Size", "VGPR_Count", "Accum_VGPR_Count", "SGPR_Count",
        "Counter_Name", "Counter_Value", "Start_Timestamp", "End_Timestamp"]


def _rows(dispatches):
    """dispatches: [(id, kernel, grid threads, duration ns, {counter: value})]"""
    out, t = [], 1_000_000
    for d, k, grid, ns, ctrs in dispatches:
        for name, v in ctrs.items():
            out.append({"Correlation_Id": d, "Dispatch_Id": d, "Agent_Id": "Agent 2", "Queue_Id": 2, "Process_Id": 1,
                        "Thread_Id": 1, "Grid_Size": grid, "Kernel_Id": 8, "Kernel_Name": k, "Workgroup_Size": 768,
                        "LDS_Block_Size": 65536, "Scratch_Size": 0, "VGPR_Count": 84, "Accum_VGPR_Count": 0,
                        "SGPR_Count": 112, "Counter_Name": name, "Counter_Value": v, "Start_Timestamp": t,
                        "End_Timestamp": t + ns})
        t += ns + 1000
    return out


def test_context_saved_dispatch_is_left_out(tmp_path):
    k = "void k_pdf_r6<0>(dprf_enum, ...)"
    grid = 256 * 768                                    # 3,072 waves
    per = 20.0                                          # bytes per candidate of the kernel's own traffic
    batch = 1 << 25
    # warm-up step (3 small launches) then two counted steps of one launch each; the second counted one was saved
    warm = [(i, k, grid, 1_000_000_000, {"WRITE_SIZE": (1 << 22) * per / 1024, "SQ_WAVES": 3072.0}) for i in (2, 4, 6)]
    counted = [(8, k, grid, 9_000_000_000, {"WRITE_SIZE": batch * per / 1024, "SQ_WAVES": 3072.0}),
               (10, k, grid, 9_000_000_000, {"WRITE_SIZE": (batch * per + 181.7e6) / 1024, "SQ_WAVES": 6144.0})]
    os.makedirs(tmp_path / "write")
    with open(tmp_path / "write" / "write_counter_collection.csv", "w", newline="") as f:
        w = csv.DictWriter(f, COLS)
        w.writeheader()
        for r in _rows(warm + counted):
            w.writerow(r)
    json.dump({"config": {"batch_per_gpu": batch, "build": "test"}, "steps": 3,
               "roofline": {"candidates_per_launch": batch}}, open(tmp_path / "bench_under_kt.json", "w"))
    out = str(tmp_path / "summary")
    subprocess.run([sys.executable, os.path.join(HERE, "..", "tools", "prof_summary.py"), str(tmp_path), out],
                   check=True, capture_output=True)
    c = json.load(open(out + ".json"))["counters"]
    (name, v), = c.items()
    assert "k_pdf_r6" in name
    saves = v["context_saves"]["write"]
    assert [s["dispatch"] for s in saves] == ["10"] and saves[0]["sq_waves"] == 6144 and saves[0]["grid_waves"] == 3072
    assert abs(v["hbm_bytes_per_candidate"] - per) < 1e-6
    assert abs(v["hbm_bytes_per_candidate_median"] - per) < 1e-6
    assert v["hbm_bytes_per_candidate_with_saves"] > per + 2.5      # the save's 181.7 MB over 2^26 candidates
    assert v["hbm_dispatch_values"]["WRITE_SIZE"] == [batch * per / 1024]   # the warm-up step is not counted
