"""bench.py --gpus N without a launcher (CPU, gloo): the parent spawns N fresh ranks with
torch.distributed.run's environment contract, hands rank 0 its CPU baseline, propagates the first
failing rank's exit code, and every rank's dist record reaches rank 0's line.  The child here is a
CPU-only stand-in for bench.py's GPU body (no engine), run through the same spawn_ranks."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

CHILD = r'''
import json, os, sys
sys.path.insert(0, {root!r})
import torch, torch.distributed as dist
import bench
assert os.environ['MASTER_ADDR'] == '127.0.0.1'
dist.init_process_group('gloo')
rec = bench.dist_record(None, torch, dist, int(os.environ['LOCAL_RANK']))
if int(os.environ['RANK']) == {fail}:
    sys.exit(3)
dist.barrier()
if dist.get_rank() == 0:
    cpu = json.load(open(os.environ[bench.CPU_FILE_ENV]))
    print('LINE ' + json.dumps(dict(dist=rec, cpu_baseline=cpu)), flush=True)
dist.destroy_process_group()
'''


def _run(tmp_path, world, fail=-1):
    script = tmp_path / 'child.py'
    script.write_text(CHILD.format(root=ROOT, fail=fail))
    out = tmp_path / 'out.txt'
    code = (f'import sys, types; sys.path.insert(0, {ROOT!r}); import bench; '
            f'a = types.SimpleNamespace(gpus={world}); '
            f'sys.exit(bench.spawn_ranks(a, {{"value": 1.0, "cores": 7}}, [sys.executable, {str(script)!r}]))')
    with open(out, 'w') as f:
        p = subprocess.run([sys.executable, '-c', code], stdout=f, stderr=subprocess.STDOUT, timeout=240,
                           env={k: v for k, v in os.environ.items() if k not in ('RANK', 'WORLD_SIZE', 'LOCAL_RANK')})
    return p.returncode, out.read_text()


@pytest.mark.timeout(300)
@pytest.mark.parametrize('world', [2, 4])
def test_spawned_ranks_form_one_group(tmp_path, world):
    rc, text = _run(tmp_path, world)
    assert rc == 0, text
    lines = [ln for ln in text.splitlines() if ln.startswith('LINE ')]
    assert len(lines) == 1, text                      # rank 0 alone prints
    rec = json.loads(lines[0][5:])
    assert rec['cpu_baseline'] == {'value': 1.0, 'cores': 7}
    d = rec['dist']
    assert d['backend'] == 'gloo' and d['world_size'] == world and d['launcher'] == 'bench.py spawn'
    assert [r['rank'] for r in d['ranks']] == list(range(world))
    assert [r['local_rank'] for r in d['ranks']] == list(range(world))


@pytest.mark.timeout(300)
def test_failing_rank_fails_the_job(tmp_path):
    rc, text = _run(tmp_path, 2, fail=1)
    assert rc == 3, (rc, text)
    assert 'LINE ' not in text


def test_bench_parent_spawns_before_any_gpu_use(monkeypatch):
    """main() with --gpus 2 and no WORLD_SIZE goes to spawn_ranks before importing torch's device
    side: the parent's only work is the CPU baseline."""
    import bench
    seen = {}
    monkeypatch.setattr(sys, 'argv', ['bench.py', '--gpus', '2', '--backend', 'gloo', '--no-cpu-baseline'])
    for k in ('WORLD_SIZE', 'RANK', 'LOCAL_RANK', bench.CPU_FILE_ENV):
        monkeypatch.delenv(k, raising=False)
    monkeypatch.setattr(bench, 'spawn_ranks', lambda args, cpu, cmd=None: seen.update(gpus=args.gpus, cpu=cpu) or 0)
    with pytest.raises(SystemExit) as ex:
        bench.main()
    assert ex.value.code == 0 and seen == {'gpus': 2, 'cpu': None}
