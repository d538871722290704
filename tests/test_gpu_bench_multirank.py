"""bench.py's multi-rank path, run for real before the driver's 8-GPU run does.

`python -m torch.distributed.run --nproc-per-node 2 bench.py --gpus 2 --dist-backend gloo --share-gpu`
launches two ranks on the one GPU of the box: process-group init, the barrier, the sharded sampler
(rank r samples its prompts with the rows of the ONE global x_T draw, /root/reference/inference.py:499-504),
the single gather, max-over-ranks timing and destroy_process_group all execute. The gathered latents of
the last timed call must equal, bitwise, a one-process run of the same global batch. Both runs are fresh
child processes; this test process never touches the GPU.
"""
import json
import os
import socket
import subprocess
import sys

import pytest

from conftest import REPO

pytestmark = pytest.mark.gpu

B = 2  # prompts per rank
COMMON = ["--steps", "1", "--warmup", "1", "--no-extra", "--cpu-baseline", "none", "--no-roofline"]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _json_line(stdout):
    lines = [ln for ln in stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, stdout[-2000:]
    return json.loads(lines[0])


def test_bench_two_ranks_gloo_matches_one_process(tmp_path):
    from safetensors.torch import load_file
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", HSA_ENABLE_IPC_MODE_LEGACY="0")
    two = tmp_path / "two.safetensors"
    one = tmp_path / "one.safetensors"
    cmd2 = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
            "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.join(REPO, "bench.py"),
            "--gpus", "2", "--batch", str(B), "--dist-backend", "gloo", "--share-gpu", "--dump-latents", str(two),
            *COMMON]
    r2 = subprocess.run(cmd2, cwd=REPO, env=env, capture_output=True, text=True, timeout=280)
    assert r2.returncode == 0, r2.stderr[-4000:]
    j2 = _json_line(r2.stdout)
    assert j2["n_gpus"] == 2 and j2["config"]["global_batch"] == 2 * B and j2["finite"] is True
    assert j2["config"]["dist_backend"] == "gloo" and j2["value"] > 0
    cmd1 = [sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "1", "--batch", str(2 * B),
            "--dump-latents", str(one), *COMMON]
    env1 = {k: v for k, v in env.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK")}
    r1 = subprocess.run(cmd1, cwd=REPO, env=env1, capture_output=True, text=True, timeout=200)
    assert r1.returncode == 0, r1.stderr[-4000:]
    j1 = _json_line(r1.stdout)
    assert j1["n_gpus"] == 1 and j1["config"]["global_batch"] == 2 * B
    lat2, lat1 = load_file(str(two))["latents"], load_file(str(one))["latents"]
    assert lat2.shape == lat1.shape == (2 * B, 640, 80)
    import torch
    assert torch.equal(lat2, lat1), float((lat2 - lat1).abs().max())
