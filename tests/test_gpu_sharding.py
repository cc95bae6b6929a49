"""The C4 multi-GPU path with the real engine: two fresh processes, one per rank,
both on cuda:0 of the one-GPU box, each running `sharding.ShardedEncodeDecode` on its shard of a
ragged batch (padded to the GLOBAL maximum, distil_codec.py:133-136) and gathering over gloo.  The
gathered codes and waveforms equal a single-process run of the whole batch bit for bit, and the
gathered rows of the first and last clip match the CPU oracle run on the same globally padded input
(codes exact on decisive frames, waveform >= 80 dB), independently of the engine."""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("lengths", [[30000, 17001, 24000, 5000, 12345], [9000, 26000]])
def test_world2_sharded_equals_single_process(cfg, state, tmp_path, lengths):
    from distilcodec_nabeel_amd import sharding, synth
    from distilcodec_nabeel_amd.engine import NativeCodec

    out = str(tmp_path / "gathered.npz")
    port = str(_free_port())
    arg = ",".join(map(str, lengths))
    procs = [subprocess.Popen([sys.executable, os.path.join(HERE, "sharded_worker.py"), str(r), "2", port, out, arg])
             for r in range(2)]
    try:
        rcs = [p.wait(timeout=240) for p in procs]
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    assert rcs == [0, 0]
    got = np.load(out)

    eng = NativeCodec(cfg, state, "cuda:0")
    audio = torch.from_numpy(sharding.pad_to_global(synth.batch_clips(lengths, 0, len(lengths), seed=3), max(lengths)))
    codes, wav = eng.encode_decode(audio.cuda())
    torch.cuda.synchronize()
    assert got["codes"].shape == tuple(codes.shape) and got["wav"].shape == tuple(wav.shape)
    assert np.array_equal(got["codes"], codes.cpu().numpy())
    assert np.array_equal(got["wav"], wav.cpu().numpy())

    from _parity import check_codes, check_wave
    from oracle import reference_cpu as R

    for i in (0, len(lengths) - 1):
        ref = R.encode_decode(audio[i: i + 1], state, cfg)
        rc = ref["codes"][0, :, :, 0].numpy()
        best, second, _ = R.top2_gap_fp64(ref["x_pjt_in"], R.codebook(state["quantizer"]))
        dec = (((second - best) / best) > 1e-4).numpy().reshape(rc.shape)
        gc = torch.from_numpy(got["codes"][i: i + 1])
        check_codes(gc, rc, dec)
        snr = check_wave(eng, gc, rc, torch.from_numpy(got["wav"][i: i + 1]), ref["wav"][:, 0].numpy(), 80)
        print(f"gathered clip {i} vs oracle: SNR {snr:.1f} dB")
