"""Recipe-depth training stays finite through many hipGraph replays.

Round 4's graphed few-shot vid2vid recipe trained to NaN within a few replays (the ROCm graph
packet-capture mode replayed the ~10^4-node iteration with stale operands; see
imaginaire_amd/__init__.py). The unit-config graph tests replay once and could not see it.
These run the few-shot vid2vid 512x512 recipe (5 downsamples, 4-frame sequences, 1 and 2
reference frames) through ``scripts/bench_families.py --graph``: 4 warm-up iterations (the
last one captures), then 8 replays; every iteration's losses must be finite (the script exits
3 otherwise) and the last replay must still have updated the networks.
Reference schedule: /root/reference/imaginaire/trainers/vid2vid.py:253-288.
"""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FS_RECIPE = [
    'gen.num_filters=32', 'gen.num_downsamples=5', 'gen.hyper.num_hyper_layers=4',
    'gen.hyper.attention.num_filters=32', 'gen.flow.num_filters=32',
    'gen.flow.max_num_filters=1024', 'gen.flow.num_res_blocks=6',
    'gen.flow.multi_spade_combine.embed.num_filters=32',
    'gen.flow.multi_spade_combine.embed.num_downsamples=5', 'gen.embed.num_filters=32',
    'gen.embed.num_downsamples=5', 'dis.image.num_filters=32', 'dis.image.max_num_filters=512',
    'dis.image.num_layers=4', 'data.train.batch_size=3',
    'data.train.augmentations.resize_h_w=512,512', 'data.val.augmentations.resize_h_w=512,512']


def _run(k):
    cmd = [sys.executable, '-u', 'scripts/bench_families.py', '--config',
           'configs/unit_test/fs_vid2vid_face.yaml', '--seq-len', '4', '--graph', '--steps', '8',
           '--warmup', '4', '--print-losses', '--set'] + FS_RECIPE + \
        ['data.initial_few_shot_K=%d' % k]
    env = dict(os.environ)
    env.pop('DEBUG_CLR_GRAPH_PACKET_CAPTURE', None)  # the package default is under test
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=110)
    return r


@pytest.mark.gpu
@pytest.mark.parametrize('k', [1, 2])
def test_fs_vid2vid_recipe_replays_stay_finite(k):
    r = _run(k)
    assert r.returncode == 0, r.stderr[-3000:]
    out = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith('{')][-1])
    assert out['hipgraph'] is True, 'the recipe iteration was not captured'
    assert out['losses_finite'] is True
    per_it = [json.loads(ln.split(' losses ', 1)[1]) for ln in r.stderr.splitlines()
              if ln.startswith('[bench_families] it ') and ' losses ' in ln]
    assert len(per_it) == 12
    for it, d in enumerate(per_it):
        for part in ('gen', 'dis'):
            for name, v in d[part].items():
                assert v == v and abs(v) != float('inf'), (it, part, name, v)
    # replays keep training: the G total moves from replay to replay
    totals = [d['gen']['total'] for d in per_it[4:]]
    assert len(set(totals)) > 1, totals
    print('fs_vid2vid recipe K=%d: %.1f frames/s (graph)' % (k, out['frames_per_s']))
