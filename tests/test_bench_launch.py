"""bench.py --gpus N outside torchrun starts N ranks itself (a torch.distributed.run child process,
no exec) and every rank joins one process group: the dry run forms the group exactly as a bench
run does (gloo here: no GPU in this container; RCCL on a GPU box) and rank 0 reports the world it
saw.  This is the launch path of the driver's 1/2/4/8-GPU scaling runs (BASELINE configs[2])."""
import json
import os
import subprocess
import sys

from conftest import ROOT


def _run(args, env_extra=None):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK",
                                                            "MASTER_ADDR", "MASTER_PORT")}
    env.update(env_extra or {})
    env["CUDA_VISIBLE_DEVICES"] = ""          # CPU-only process group even on a GPU box
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, env=env, cwd="/tmp",
                       capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout            # rank 0 alone prints, exactly one JSON line
    return json.loads(lines[0]), p.stderr


def test_bench_gpus_n_launches_n_ranks():
    out, err = _run(["--gpus", "2", "--dry-run"])
    assert "launching 2 ranks" in err
    assert out["n_gpus"] == 2 and out["dist"]["world_size"] == 2
    assert out["dist"]["backend"] == "gloo"
    assert out["global_batch"] == 32             # bs 16 per rank


def test_bench_single_gpu_runs_in_process():
    out, err = _run(["--dry-run"])
    assert "launching" not in err
    assert out["n_gpus"] == 1 and out["dist"]["world_size"] == 1
