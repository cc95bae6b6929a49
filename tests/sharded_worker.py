"""One rank of the world-size-2 sharded encode -> decode test (tests/test_gpu_sharding.py), run as a
fresh process: `python tests/sharded_worker.py RANK WORLD PORT OUT LEN,LEN,...`.  Both ranks share
cuda:0 (one GPU box) and gather over gloo; rank 0 writes the gathered codes and waveforms to OUT."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    rank, world, port, out = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3], sys.argv[4]
    lengths = [int(x) for x in sys.argv[5].split(",")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=port)
    import numpy as np
    import torch
    import torch.distributed as dist

    from distilcodec_nabeel_amd import config, sharding, synth, weights
    from distilcodec_nabeel_amd.engine import NativeCodec

    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        cfg = config.default_config()
        eng = NativeCodec(cfg, weights.synthetic_state_dict(cfg, seed=1234), "cuda:0")
        s, e = sharding.shard_bounds(len(lengths), rank, world)
        run = sharding.ShardedEncodeDecode(eng, synth.batch_clips(lengths, s, e, seed=3), max(lengths), len(lengths),
                                           rank, world)
        codes, _ = run.step()
        wav = run.gather_wav()
        torch.cuda.synchronize()
        if rank == 0:
            np.savez(out, codes=codes.cpu().numpy(), wav=wav.cpu().numpy())
        dist.barrier()
    finally:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
