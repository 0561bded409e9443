"""TunableOp A/B for the library GEMMs (hipBLASLt / rocBLAS): tune every GEMM shape of one 8-frame bf16
edit with WARM operands (rotating buffer 0: the pipeline's GEMM inputs were just written by the previous
kernel), write the table, then time edits with the table against hipBLASLt's own heuristic.

  python tools/tune_gemms.py OUT.csv      (GPU box)"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    out = os.path.abspath(sys.argv[1])
    if len(sys.argv) > 2 and sys.argv[2] == "tune":
        import torch
        torch.cuda.tunable.enable(True)
        torch.cuda.tunable.tuning_enable(True)
        torch.cuda.tunable.set_rotating_buffer_size(0)
        torch.cuda.tunable.set_max_tuning_duration(20)
        torch.cuda.tunable.set_filename(out, insert_device_ordinal=False)
        sys.argv = ["bench.py", "--steps", "1", "--warmup", "0", "--extras", "none", "--no-cpu-baseline", "--no-events"]
        sys.path.insert(0, ROOT)
        import bench
        bench.main()
        torch.cuda.tunable.write_file()
        return
    subprocess.run([sys.executable, __file__, out, "tune"], check=True, cwd=ROOT)
    res = {}
    for mode in ("heuristic", "table", "heuristic", "table"):
        env = dict(os.environ)
        if mode == "table":
            env.update(PYTORCH_TUNABLEOP_ENABLED="1", PYTORCH_TUNABLEOP_TUNING="0", PYTORCH_TUNABLEOP_FILENAME=out)
        r = subprocess.run([sys.executable, "bench.py", "--steps", "2", "--warmup", "1", "--extras", "none",
                            "--no-cpu-baseline", "--no-events"], cwd=ROOT, env=env, capture_output=True, text=True,
                           check=True)
        d = json.loads(r.stdout.strip().splitlines()[-1])
        res.setdefault(mode, []).append(d["ms_per_step"])
        print(json.dumps({"mode": mode, "ms_per_edit": d["ms_per_step"], "frames_per_s": d["value"]}), flush=True)


if __name__ == "__main__":
    main()
