"""One rank of the real-engine sharded encode (tests/test_sharding.py::test_sharded_real_engines_match_single).

Run under ``torch.distributed.run --nproc-per-node 2``: every rank builds its own HIP engine (on cuda:0 --
the test box has one GPU; on a node, LOCAL_RANK's GPU), joins a gloo group, and encodes its round-robin share
through ``DistributedMimiEncoder``; rank 0 writes the merged codes to the .npz named on the command line.
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "tokenize-audio_amd"), ROOT):
    sys.path.insert(0, p)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from mimi_hip import synthetic  # noqa: E402
from mimi_hip.encoder import MimiEncoder  # noqa: E402
from mimi_hip.model import MimiHipModel  # noqa: E402
from mimi_hip.sharding import DistributedMimiEncoder  # noqa: E402

N_CLIPS, BATCH = 11, 3


def clips():
    lengths = synthetic.random_lengths(N_CLIPS, 0.2, 3.0, seed=5)
    return [synthetic.speech_like(L, 5, i) for i, L in enumerate(lengths)]


def main(out_path):
    dist.init_process_group("gloo")
    try:
        ndev = torch.cuda.device_count()
        dev = f"cuda:{int(os.environ.get('LOCAL_RANK', '0')) % ndev}"
        torch.cuda.set_device(dev)
        model = MimiHipModel(synthetic.make_state_dict(seed=0), device=dev)
        enc = DistributedMimiEncoder(encoder=MimiEncoder(device=dev, model=model), batch_size=BATCH)
        out = enc.encode_all(clips())
        if dist.get_rank() == 0:
            np.savez(out_path, **{f"c{i}": c for i, c in enumerate(out)})
        model.close()
    finally:
        dist.destroy_process_group()


if __name__ == "__main__":
    main(sys.argv[1])
