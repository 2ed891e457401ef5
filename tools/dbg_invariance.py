"""Debug: which stage breaks batch invariance (row i alone vs inside a batch)."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from adaptive_amd import Config, Encoder2Decoder, synth
dev = torch.device("cuda:0")
m = Encoder2Decoder(Config()).to(dev).load_synthetic(123)
feats = torch.from_numpy(synth.make_features(300, seed=11)).to(dev)
full = m._encode(feats)
names = ["V", "v_g", "h0c0", "a_g", "VWv"]
for lo, hi in [(0, 1), (37, 74), (250, 300)]:
    part = m._encode(feats[lo:hi].contiguous())
    for n, a, b in zip(names, full, part):
        if n == "h0c0":
            print(lo, hi, "h0", torch.equal(a[0][lo:hi], b[0]), "c0", torch.equal(a[1][lo:hi], b[1]))
        else:
            print(lo, hi, n, torch.equal(a[lo:hi], b), (a[lo:hi] - b).abs().max().item())
    caps = torch.full((300, 1), 1, dtype=torch.int64, device=dev)
    sf = m.decoder(full[0], full[1], caps, full[2])
    sp = m.decoder(part[0], part[1], caps[lo:hi], part[2])
    for n, a, b in zip(["scores", "alpha", "beta"], sf[:3], sp[:3]):
        print(lo, hi, n, torch.equal(a[lo:hi], b), (a[lo:hi] - b).abs().max().item())
    print(lo, hi, "h", torch.equal(sf[3][0][:, lo:hi], sp[3][0]), "c", torch.equal(sf[3][1][:, lo:hi], sp[3][1]))
