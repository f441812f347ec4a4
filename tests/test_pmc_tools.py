"""CPU: the profile summarisers keep counters tied to the build they counted: a VALU mix whose
passes profiled another build than the PMC summary it is paired with is refused (tools/pmc_mix_summary.py)."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TOOL = os.path.join(ROOT, "tools", "pmc_mix_summary.py")
COUNTERS = {"mix1": ["SQ_INSTS_VALU", "SQ_INSTS_VALU_ADD_F32", "SQ_INSTS_VALU_MUL_F32"],
            "mix2": ["SQ_INSTS_VALU_FMA_F32", "SQ_INSTS_VALU_INT32"]}


def _passes(d, ids):
    for (p, names), kid in zip(COUNTERS.items(), ids):
        os.makedirs(d / p)
        rows = ["Dispatch_Id,Kernel_Name,Counter_Name,Counter_Value,Start_Timestamp,End_Timestamp"]
        rows += [f"1,sail_trace_kernel_jit,{n},{1000 * (i + 1)},0,5000" for i, n in enumerate(names)]
        (d / p / "run_counter_collection.csv").write_text("\n".join(rows) + "\n")
        (d / (p + ".log")).write_text(json.dumps({"roofline": {"kernel_id": kid}}) + "\n")


def _summary(path, kid, spp=64):
    path.write_text(json.dumps({"kernel_id": kid, "workload": "w", "launch": {"pixels": 16, "spp": spp, "bounces": 8}}))
    return str(path)


def _run(d, out, *extra):
    return subprocess.run([sys.executable, TOOL, str(d), str(out), "16", "64", "8", "w", *extra],
                          capture_output=True, text=True)


def test_mix_paired_with_the_same_build(tmp_path):
    _passes(tmp_path / "m", ["k@1", "k@1"])
    r = _run(tmp_path / "m", tmp_path / "o.json", "100", _summary(tmp_path / "s.json", "k@1"))
    assert r.returncode == 0, r.stderr
    rec = json.loads((tmp_path / "o.json").read_text())
    assert rec["kernel_id"] == "k@1" and rec["paired_summary"] == "s.json"


def test_mix_of_another_build_or_shape_refused(tmp_path):
    _passes(tmp_path / "m", ["k@1", "k@1"])
    for i, summ in enumerate([_summary(tmp_path / "a.json", "k@2"), _summary(tmp_path / "b.json", "k@1", spp=1024)]):
        out = tmp_path / f"o{i}.json"
        r = _run(tmp_path / "m", out, "100", summ)
        assert r.returncode == 2 and "refused" in r.stderr and not out.exists()


def test_mix_passes_of_two_builds_refused(tmp_path):
    _passes(tmp_path / "m", ["k@1", "k@2"])
    r = _run(tmp_path / "m", tmp_path / "o.json")
    assert r.returncode != 0 and not (tmp_path / "o.json").exists()
