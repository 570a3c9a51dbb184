"""bench.py's launcher contract on the CPU: `--gpus N` is the job's rank
count. More ranks than the box has GPUs, or a launcher world size that
disagrees with --gpus, exits non-zero before touching a GPU -- never a
silent single-GPU line."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, env_extra=None):
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    env.update(env_extra or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, env=env, capture_output=True,
                          text=True, timeout=300)


def test_more_gpus_than_the_box_has_fails():
    import torch
    n = torch.cuda.device_count()  # counting does not initialise a GPU
    r = _run(["--gpus", str(n + 1), "--steps", "1", "--warmup", "0"])
    assert r.returncode != 0
    assert "GPU" in r.stderr and '"metric"' not in r.stdout


def test_world_size_disagreeing_with_gpus_fails():
    r = _run(["--gpus", "2"], {"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode != 0
    assert "WORLD_SIZE=1" in r.stderr and '"metric"' not in r.stdout


def test_gpus_must_be_positive():
    r = _run(["--gpus", "0"])
    assert r.returncode != 0 and '"metric"' not in r.stdout


def test_evidence_lookup_follows_latest():
    """The roofline's traffic and trace figures come from the evidence
    directory profiles/LATEST names (a path under profiles/), and the line
    says so (`latest`: true) -- for the compaction and the cfg4 tally kernel."""
    import importlib.util
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    b = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(b)
    latest = b.latest_dir()
    assert latest is not None and os.path.isdir(latest)
    assert b.evidence_dirs()[0] == latest
    for kernel, cfg in (("place_compact_kernel", 2), ("tally_wave1_kernel", 4)):
        t = b.pmc_traffic(kernel, cfg)
        assert t is not None and t["latest"], (kernel, t)
