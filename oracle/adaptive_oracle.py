"""CPU oracle for the adaptive-attention greedy decode — TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import
this module, and only as the checker / the timed CPU baseline.  The product path
(``adaptive_amd``) never calls it and fails loudly when its HIP library is missing.

What it is: a PyTorch-CPU fp32 restatement of the reference's ``Encoder2Decoder.sampler``
(``code_src/models/adaptive_attention.py:168-216``), op for op and in the reference's order,
including its redundant work (``W_v V`` recomputed every step, ``W_g h`` computed twice, the
``W_h * 0`` sentinel term), so that it is also the honest CPU baseline.  Two deliberate deviations,
both documented in SURVEY.md §3:

* D1 — ``adaptive_attention.sampler`` feeds ``(h0, c0)`` of shape [B,1,H] straight into
  ``nn.LSTM`` (``adaptive_attention.py:183,198``), which raises for B > 1.  The oracle applies the
  baseline sampler's transpose (``baseline_attention.py:251-252``) — the intended semantics; for
  B = 1 the tokens are unchanged.
* D2 — irrelevant here (training only).

Pinning: ``tests/golden/make_golden.py`` imports the real reference modules (torchvision stubbed,
ResNet trunk = identity) in the survey container and records its outputs; ``tests/test_oracle.py``
checks this restatement against those fixtures.
"""
from __future__ import annotations

from typing import Dict, Tuple

import numpy as np
import torch
import torch.nn.functional as F

ATT = 49  # attention width / spatial locations (adaptive_attention.py:16-19)


class OracleModel:
    """Holds fp32 CPU tensors keyed like the reference state dict."""

    def __init__(self, state: Dict[str, np.ndarray]):
        self.w = {k: torch.from_numpy(np.ascontiguousarray(v)).float() for k, v in state.items()}
        H = self.w["decoder.LSTM.weight_hh_l0"].shape[1]
        In = self.w["decoder.LSTM.weight_ih_l0"].shape[1]
        # nn.LSTM(embed*2, hidden, 1, batch_first=True)  (baseline_attention.py:140)
        self.lstm = torch.nn.LSTM(In, H, 1, batch_first=True)
        with torch.no_grad():
            for n in ("weight_ih_l0", "weight_hh_l0", "bias_ih_l0", "bias_hh_l0"):
                getattr(self.lstm, n).copy_(self.w["decoder.LSTM." + n])
        self.lstm.eval()
        self.lstm.requires_grad_(False)

    # ---- AttentiveCNN.forward tail (baseline_attention.py:36-62), trunk = identity -------------
    def encoder(self, A: torch.Tensor):
        w = self.w
        B = A.size(0)
        a_g = F.avg_pool2d(A, 7)                                   # :46  nn.AvgPool2d(7)
        a_g = a_g.view(B, -1)                                      # :47
        V = A.view(B, A.size(1), -1).transpose(1, 2)               # :50
        V = F.relu(F.linear(V, w["encoder.affine_a.weight"], w["encoder.affine_a.bias"]))   # :51
        v_g = F.relu(F.linear(a_g, w["encoder.affine_b.weight"], w["encoder.affine_b.bias"]))  # :53
        h0 = torch.tanh(F.linear(a_g, w["encoder.affine_h0.weight"], w["encoder.affine_h0.bias"])).unsqueeze(1)  # :56-57
        c0 = torch.tanh(F.linear(a_g, w["encoder.affine_c0.weight"], w["encoder.affine_c0.bias"])).unsqueeze(1)  # :58-59
        # D1: baseline_attention.py:251-252 transposes states to [1,B,H] before the LSTM
        return V, v_g, (h0.transpose(0, 1), c0.transpose(0, 1)), a_g

    # ---- Atten.forward (adaptive_attention.py:26-58) --------------------------------------------
    def atten(self, V, h_t, s_t):
        w = self.w
        Wv = w["decoder.adaptive.atten.affine_v.weight"]
        Wg = w["decoder.adaptive.atten.affine_g.weight"]
        Ws = w["decoder.adaptive.atten.affine_s.weight"]
        wh = w["decoder.adaptive.atten.affine_h.weight"]
        content_v = F.linear(V, Wv).unsqueeze(1) + F.linear(h_t, Wg).unsqueeze(2)          # :34-35
        z_t = F.linear(torch.tanh(content_v), wh).squeeze(3)                               # :38
        alpha_t = F.softmax(z_t.view(-1, z_t.size(2)), dim=1).view(z_t.size(0), z_t.size(1), -1)  # :39
        c_t = torch.bmm(alpha_t, V).squeeze(2)                                             # :42
        content_s = F.linear(s_t, Ws) + F.linear(h_t, Wg)                                  # :45
        z_t_extended = F.linear(torch.tanh(content_s), wh)                                 # :47
        extended = torch.cat((z_t, z_t_extended), dim=2)                                   # :50
        alpha_hat_t = F.softmax(extended.view(-1, extended.size(2)), dim=1).view(extended.size(0), extended.size(1), -1)  # :51
        beta_t = alpha_hat_t[:, :, -1].unsqueeze(2)                                         # :52-55
        c_hat_t = beta_t * s_t + (1 - beta_t) * c_t                                         # :56
        return c_hat_t, alpha_t, beta_t

    # ---- AdaptiveBlock.forward (adaptive_attention.py:110-134) ----------------------------------
    def adaptive(self, x, hiddens, cells, V):
        w = self.w
        B, H = x.size(0), hiddens.size(2)
        h0 = torch.zeros(1, B, H).transpose(0, 1)                                           # :116 init_hidden
        if hiddens.size(1) > 1:
            hiddens_t_1 = torch.cat((h0, hiddens[:, :-1, :]), dim=1)                        # :120
        else:
            hiddens_t_1 = h0                                                                # :122
        # Sentinel.forward (:75-85)
        gate = F.linear(x, w["decoder.adaptive.sentinel.affine_x.weight"]) + \
            F.linear(hiddens_t_1, w["decoder.adaptive.sentinel.affine_h.weight"])
        sentinel = torch.sigmoid(gate) * torch.tanh(cells)
        c_hat, alpha, beta = self.atten(V, hiddens, sentinel)                               # :128
        scores = F.linear(c_hat + hiddens, w["decoder.adaptive.mlp.weight"], w["decoder.adaptive.mlp.bias"])  # :132
        return scores, alpha, beta

    # ---- Decoder.forward (baseline_attention.py:148-194) ----------------------------------------
    def decoder(self, V, v_g, captions, states):
        w = self.w
        embeddings = F.embedding(captions, w["decoder.embed.weight"])                      # :151
        x = torch.cat((embeddings, v_g.unsqueeze(1).expand_as(embeddings)), dim=2)         # :154
        H = self.lstm.hidden_size
        hiddens = torch.zeros(x.size(0), x.size(1), H)                                      # :161-163
        cells = torch.zeros(x.size(1), x.size(0), H)
        for time_step in range(x.size(1)):                                                  # :167
            x_t = x[:, time_step, :].unsqueeze(1)
            h_t, states = self.lstm(x_t, states)                                            # :172
            hiddens[:, time_step, :] = h_t.squeeze(1)
            cells[time_step, :, :] = states[1]
        cells = cells.transpose(0, 1)                                                       # :181
        scores, alpha, beta = self.adaptive(x, hiddens, cells, V)                           # :189
        return scores, alpha, beta, states

    # ---- Encoder2Decoder.sampler (adaptive_attention.py:168-216) --------------------------------
    @torch.no_grad()
    def sampler(self, images: torch.Tensor, max_len: int = 30, keep_scores: bool = False):
        V, v_g, states, _ = self.encoder(images)
        captions = torch.LongTensor(images.size(0), 1).fill_(1)                            # :190 <start>=1
        sampled_ids, attention, Beta, all_scores = [], [], [], []
        for _ in range(max_len):                                                            # :197
            scores, atten_weights, beta, states = self.decoder(V, v_g, captions, states)
            predicted = scores.max(2)[1]                                                    # :201
            captions = predicted
            sampled_ids.append(captions)
            attention.append(atten_weights)
            Beta.append(beta)
            if keep_scores:
                all_scores.append(scores)
        out = (torch.cat(sampled_ids, dim=1), torch.cat(attention, dim=1), torch.cat(Beta, dim=1))
        if keep_scores:
            return out + (torch.cat(all_scores, dim=1),)
        return out


def top2_margin(scores: torch.Tensor) -> torch.Tensor:
    """top1 - top2 logit per (row, step): how much error an argmax can absorb."""
    t = scores.topk(2, dim=-1).values
    return t[..., 0] - t[..., 1]


def sampler(state: Dict[str, np.ndarray], feats: np.ndarray, max_len: int = 20, keep_scores: bool = False):
    """numpy in / torch out convenience wrapper."""
    m = OracleModel(state)
    return m.sampler(torch.from_numpy(np.ascontiguousarray(feats)), max_len=max_len, keep_scores=keep_scores)


class TrainOracle(OracleModel):
    """Teacher-forced ``Encoder2Decoder.forward`` (``baseline_attention.py:206-230``) with autograd:
    every reference parameter is a leaf tensor with ``requires_grad`` (``self.w``), the LSTM is an
    ``nn.LSTM`` whose parameters are those leaves.  D2 is moot here: the states
    are transposed out of place.  Returns the packed scores like ``pack_padded_sequence``."""

    def __init__(self, state: Dict[str, np.ndarray]):
        super().__init__(state)
        for v in self.w.values():
            v.requires_grad_(True)
        self.lstm.train()
        self.lstm.requires_grad_(True)
        with torch.no_grad():  # the LSTM module's own parameters ARE the leaves of self.w
            for n in ("weight_ih_l0", "weight_hh_l0", "bias_ih_l0", "bias_hh_l0"):
                setattr(self.lstm, n, torch.nn.Parameter(self.w["decoder.LSTM." + n]))
        for n in ("weight_ih_l0", "weight_hh_l0", "bias_ih_l0", "bias_hh_l0"):
            self.w["decoder.LSTM." + n] = getattr(self.lstm, n)
        self.lstm.flatten_parameters()

    def forward(self, images: torch.Tensor, captions: torch.Tensor, lengths):
        from torch.nn.utils.rnn import pack_padded_sequence
        V, v_g, states, _ = self.encoder(images)                                    # :213-219
        scores, _, _, _ = self.decoder(V, v_g, captions, states)                      # :225
        return pack_padded_sequence(scores, list(lengths), batch_first=True)        # :228

    def loss(self, images, captions, lengths):
        """train.py:101,204-208: CE over the packed scores against the packed next tokens."""
        from torch.nn.utils.rnn import pack_padded_sequence
        packed = self.forward(images, captions, lengths)
        targets = pack_padded_sequence(captions[:, 1:], list(lengths), batch_first=True)[0]
        return torch.nn.functional.cross_entropy(packed[0], targets), packed


class BeamOracle(OracleModel):
    """Beam-search decode — BUILD-DEFINED semantics (the reference has no beam search:
    ``for_wzn:3`` lists it as a TODO), so this restatement *is* the
    specification that ``aa_beam_decode`` is tested against (parity unpinned by the reference).

    Each step runs the reference's own decoder step (``Decoder.forward`` with one token,
    ``adaptive_attention.py:198``, states transposed as in D1) on the B*K hypothesis rows
    (row b*K + k, image-major), then: ``logp = log_softmax(scores)``; candidate = parent's
    cumulative score + logp; at step 0 only beam 0 is live; a finished beam (emitted ``end_id``)
    contributes the single candidate ``end_id`` at its unchanged score; the K best candidates per
    image (score descending, ties to the smaller ``k*V + v`` — a stable sort) survive.  All
    ``max_len`` steps run; final beams come out best first."""

    @torch.no_grad()
    def beam_search(self, images: torch.Tensor, max_len: int = 20, beam_size: int = 3, end_id: int = 2,
                    return_margin: bool = False, return_steps: bool = False):
        """-> ids [B,T], alpha [B,T,49], beta [B,T,1], seqs [B,K,T], scores [B,K] (+ margin: the
        smallest gap, over images and steps, between consecutive candidates among the K+1 best —
        how much score error the selection and its order can absorb; + with ``return_steps`` a list
        over steps of (per-image smallest such gap [B], the K surviving cumulative scores [B,K]))."""
        K = beam_size
        margin = float("inf")
        steps = []
        V, v_g, (h, c), _ = self.encoder(images)
        B = images.size(0)
        Vk = V.repeat_interleave(K, 0)
        vgk = v_g.repeat_interleave(K, 0)
        states = (h.repeat_interleave(K, 1), c.repeat_interleave(K, 1))
        nv = self.w["decoder.adaptive.mlp.weight"].shape[0]
        tok = torch.ones(B * K, 1, dtype=torch.long)                               # <start> = 1
        cum = torch.zeros(B, K)
        fin = torch.zeros(B, K, dtype=torch.bool)
        htok, hpar, hal, hbe = [], [], [], []
        base = (torch.arange(B) * K).unsqueeze(1)
        for t in range(max_len):
            scores, alpha, beta, states = self.decoder(Vk, vgk, tok, states)
            logp = F.log_softmax(scores[:, 0, :], dim=1).view(B, K, nv)
            cand = cum.unsqueeze(2) + logp
            if t == 0:
                cand[:, 1:, :] = -float("inf")
            if end_id >= 0 and fin.any():
                bb, kk = fin.nonzero(as_tuple=True)
                cand[bb, kk, :] = -float("inf")
                cand[bb, kk, end_id] = cum[bb, kk]
            vals, idx = torch.sort(cand.view(B, K * nv), dim=1, descending=True, stable=True)
            top = vals[:, :K + 1]
            gaps = top[:, :-1] - top[:, 1:]
            per_img = torch.where(torch.isfinite(gaps), gaps, torch.full_like(gaps, float("inf"))).min(1).values
            gaps = gaps[torch.isfinite(gaps)]
            if gaps.numel():
                margin = min(margin, float(gaps.min()))
            vals, idx = vals[:, :K], idx[:, :K]
            steps.append((per_img, vals.clone()))
            parent, token = idx // nv, idx % nv
            cum = vals
            fin = fin.gather(1, parent) | ((token == end_id) if end_id >= 0 else torch.zeros_like(fin))
            rows = (base + parent).view(-1)
            states = (states[0][:, rows], states[1][:, rows])
            tok = token.reshape(B * K, 1)
            htok.append(token)
            hpar.append(parent)
            hal.append(alpha[:, 0].view(B, K, -1))
            hbe.append(beta[:, 0, 0].view(B, K))
        T = max_len
        seqs = torch.zeros(B, K, T, dtype=torch.long)
        ids = torch.zeros(B, T, dtype=torch.long)
        al = torch.zeros(B, T, hal[0].size(2)) if T else torch.zeros(B, 0, ATT)
        be = torch.zeros(B, T, 1)
        j = torch.arange(K).expand(B, K).clone()
        for t in range(T - 1, -1, -1):
            seqs[:, :, t] = htok[t].gather(1, j)
            p = hpar[t].gather(1, j)
            al[:, t] = hal[t][torch.arange(B), p[:, 0]]
            be[:, t, 0] = hbe[t][torch.arange(B), p[:, 0]]
            j = p
        ids = seqs[:, 0].clone()
        out = (ids, al, be, seqs, cum) + ((margin,) if return_margin else ()) + ((steps,) if return_steps else ())
        return out
