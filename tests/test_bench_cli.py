"""bench.py's launcher logic on the CPU (no GPU is touched): `--gpus N`
started directly spawns its own N ranks under torch.distributed.run (the
driver's 1/2/4/8-GPU scaling runs need no external launcher); inside a rank
(WORLD_SIZE set) it never spawns again."""
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import bench  # noqa: E402  (imports numpy only at module level)


def test_needs_spawn():
    assert bench.needs_spawn(8, {})
    assert bench.needs_spawn(2, {"RANK": "0"})
    assert not bench.needs_spawn(1, {})
    assert not bench.needs_spawn(8, {"WORLD_SIZE": "8"})  # a rank of the launcher


def test_launcher_cmd_is_the_single_node_launcher():
    cmd = bench.launcher_cmd(4, 29512, ["--gpus", "4", "--steps", "20", "--warmup", "5"])
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nnodes=1" in cmd and "--nproc-per-node=4" in cmd
    assert "--master-addr=127.0.0.1" in cmd and "--master-port=29512" in cmd
    i = cmd.index(os.path.join(REPO, "bench.py"))
    assert cmd[i + 1:] == ["--gpus", "4", "--steps", "20", "--warmup", "5"]


def test_spawned_ranks_run_and_exit_status_propagates(tmp_path):
    """spawn_ranks starts torch.distributed.run with 2 ranks of a stand-in
    script (the real bench needs a GPU); every rank sees WORLD_SIZE / RANK /
    MASTER_ADDR=127.0.0.1, and a failing rank's status comes back."""
    script = tmp_path / "rank.py"
    script.write_text("import os, sys\n"
                      "open(os.path.join(os.path.dirname(__file__), 'r%s' % os.environ['RANK']), 'w').write(\n"
                      "    os.environ['WORLD_SIZE'] + ' ' + os.environ['MASTER_ADDR'])\n"
                      "sys.exit(int(os.environ.get('FAIL_RANK', '-1')) == int(os.environ['RANK']))\n")
    code = ("import sys, bench; bench.launcher_cmd = lambda g, p, argv: [sys.executable, '-m', "
            "'torch.distributed.run', '--nnodes=1', f'--nproc-per-node={g}', '--master-addr=127.0.0.1', "
            f"f'--master-port={{p}}', {str(script)!r}, *argv]; sys.exit(bench.spawn_ranks(2, []))")
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, "-c", code], cwd=REPO, env=env, timeout=240)
    assert r.returncode == 0
    assert sorted(p.name for p in tmp_path.iterdir() if p.name.startswith("r")) == ["r0", "r1", "rank.py"]
    assert (tmp_path / "r0").read_text() == "2 127.0.0.1"
    env["FAIL_RANK"] = "1"
    r = subprocess.run([sys.executable, "-c", code], cwd=REPO, env=env, timeout=240)
    assert r.returncode != 0
