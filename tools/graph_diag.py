"""Round-6 diagnostic: GraphedHop replays against eager encode_decode, per h3 switch set."""
import os, sys
import numpy as np
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distilcodec_nabeel_amd import config, weights, synth
from distilcodec_nabeel_amd.engine import NativeCodec
from distilcodec_nabeel_amd.streaming import GraphedHop

cfg = config.default_config()
state = weights.synthetic_state_dict(cfg, seed=1234)
eng = NativeCodec(cfg, state, "cuda:0")
audio = np.concatenate(synth.clips(1, 24000 * 3, seed=9, kind="speech"))
chunks = [torch.from_numpy(audio[i * 24000:(i + 1) * 24000].astype(np.float32)).cuda()[None] for i in range(3)]
for name, kn in [("x6", dict(DCX_H3=0, DCX_H3_PAIRS=0, DCX_H3_1X1=0)), ("h3 1x1 only", dict(DCX_H3=0, DCX_H3_PAIRS=0)),
                 ("h3 wide only", dict(DCX_H3_PAIRS=0, DCX_H3_1X1=0)), ("h3 pairs only", dict(DCX_H3=0, DCX_H3_1X1=0)),
                 ("all", {})]:
    with eng.knobs(**kn):
        hop = GraphedHop(eng, 24000)
        res = []
        for rep in range(2):
            for c in chunks:
                _, w0 = eng.encode_decode(torch.nn.functional.pad(c, (1, 0)))
                w0 = w0.clone()
                _, gw = hop(c)
                torch.cuda.synchronize()
                res.append(float((gw - w0).abs().max()))
    print(f"{name}: max |replay - eager| per call {['%.3g' % r for r in res]}", flush=True)
