"""Generate golden vectors by running the REAL reference ``Encoder2Decoder.sampler`` on CPU.

Run in the survey/build container only (``/root/reference`` does not exist on the GPU box):

    python tests/golden/make_golden.py [case ...]

How the reference is driven:
* ``torchvision`` is absent: a stub module whose ``resnet152`` returns an empty ``nn.Module``, so
  ``AttentiveCNN`` (``code_src/models/baseline_attention.py:16-18``) builds ``resnet_conv`` as an
  empty ``nn.Sequential`` == identity and ``images`` are post-trunk features [B,2048,7,7].
* Weights: ``adaptive_amd.synth.make_weights`` loaded with ``load_state_dict(strict=True)``.
* D1 (``adaptive_attention.py:183,198`` feeds [B,1,H] states to ``nn.LSTM``): the encoder's states
  are transposed to [1,B,H] as ``baseline_attention.py:251-252`` does.
* ``sys.dont_write_bytecode`` keeps the read-only reference tree untouched.

Outputs are data only (inputs are regenerated from seeds, their sha256 is recorded).
"""
from __future__ import annotations

import json
import os
import sys
import types

sys.dont_write_bytecode = True
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from adaptive_amd import synth  # noqa: E402

REF = "/root/reference"


def load_reference():
    tv = types.ModuleType("torchvision")
    tvm = types.ModuleType("torchvision.models")
    tvm.resnet152 = lambda pretrained=False: torch.nn.Module()  # no children -> identity trunk
    tv.models = tvm
    sys.modules["torchvision"] = tv
    sys.modules["torchvision.models"] = tvm
    sys.path.insert(0, REF)
    from code_src.models import adaptive_attention  # noqa: E402
    return adaptive_attention


class Cf:
    adaptive_word_embed_size = 256
    adaptive_lstm_hidden_size = 512
    vocab_length = 10123


def build(aa, state):
    torch.manual_seed(0)
    m = aa.Encoder2Decoder(Cf())
    m.load_state_dict({k: torch.from_numpy(v) for k, v in state.items()}, strict=True)
    m.eval()
    enc_forward = m.encoder.forward

    def enc_fixed(images):  # D1: baseline_attention.py:251-252 semantics
        V, v_g, (h0, c0) = enc_forward(images)
        return V, v_g, (h0.transpose(0, 1), c0.transpose(0, 1))

    m.encoder.forward = enc_fixed
    return m


def run(m, feats, T, scores_hook=False):
    """sampler() plus per-step logits captured by wrapping decoder.forward."""
    logs = []
    dec_forward = m.decoder.forward

    def dec_spy(*a, **k):
        out = dec_forward(*a, **k)
        logs.append(out[0].detach().clone())
        return out

    m.decoder.forward = dec_spy
    with torch.no_grad():
        ids, alpha, beta = m.sampler(torch.from_numpy(feats), max_len=T)
    m.decoder.forward = dec_forward
    scores = torch.cat(logs, dim=1)  # [B,T,V]
    top2 = scores.topk(2, dim=-1).values
    margin = (top2[..., 0] - top2[..., 1]).numpy()
    return ids.numpy(), alpha.numpy(), beta.numpy(), scores.numpy(), margin


def main(only=None):
    torch.set_num_threads(8)
    aa = load_reference()
    manifest = {"reference": "wzn0828/Adaptive code_src/models/adaptive_attention.py Encoder2Decoder.sampler",
                "torch": torch.__version__, "T": 20, "cases": {}}
    T = 20
    cases = [
        # name, weight seed, bias_noise, feature seed, B, what to keep
        ("ref_b4", 123, 0.0, 0, 4, "full"),
        ("ref_b64", 123, 0.0, 0, 64, "alpha"),
        ("ref_b512", 123, 0.0, 0, 512, "ids"),
        ("biased_b16", 99, 0.02, 5, 16, "full"),
    ]
    if only:  # regenerate some cases only; the manifest keeps the others' entries
        with open(os.path.join(HERE, "manifest.json")) as f:
            manifest["cases"] = json.load(f)["cases"]
    for name, wseed, noise, fseed, B, keep in cases:
        if only and name not in only:
            continue
        state = synth.make_weights(wseed, bias_noise=noise)
        feats = synth.make_features(B, seed=fseed)
        m = build(aa, state)
        ids, alpha, beta, scores, margin = run(m, feats, T)
        out = {"ids": ids.astype(np.int16), "beta": beta.astype(np.float32), "margin": margin.astype(np.float32)}
        if keep in ("full", "alpha"):
            out["alpha"] = alpha.astype(np.float32)
        if keep == "ids":  # alpha of every 4th row (each 64-row tile of the decode kernels sampled)
            out["alpha_s4"] = alpha[::4].astype(np.float32)
        if keep == "full":
            # full logits of rows 0,1 at steps 0,1 and step-0 logits of every row
            out["scores_r01_t01"] = scores[:2, :2].astype(np.float32)
            out["scores_t0"] = scores[:, 0].astype(np.float32)
        np.savez_compressed(os.path.join(HERE, f"{name}.npz"), **out)
        manifest["cases"][name] = {
            "weight_seed": wseed, "bias_noise": noise, "feature_seed": fseed, "B": B,
            "weights_sha256": synth.digest(state), "features_sha256": synth.digest({"f": feats})["f"],
            "min_margin": float(margin.min()), "margins_below_1e-4": int((margin < 1e-4).sum()),
            "distinct_tokens": int(len(np.unique(ids))),
        }
        print(name, manifest["cases"][name]["min_margin"], manifest["cases"][name]["margins_below_1e-4"],
              manifest["cases"][name]["distinct_tokens"])
    # module surface the drop-in must mirror
    m = build(aa, synth.make_weights(123))
    manifest["state_dict"] = {k: list(v.shape) for k, v in m.state_dict().items()}
    with open(os.path.join(HERE, "manifest.json"), "w") as f:
        json.dump(manifest, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main(sys.argv[1:])  # optional case names
