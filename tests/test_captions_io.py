"""CPU: caption post-processing and checkpoint I/O around the decode:
id -> word sentences as the reference's coco_eval builds them (code_src/tools/utils.py:176-193),
the vocabulary wrapper (code_src/data/build_vocab.py:9-28), and state-dict checkpoints in the
reference's naming and key format (train.py:177-178, model_factory.py:15-20)."""
import json

import numpy as np
import pytest
import torch

from adaptive_amd import Config, Encoder2Decoder
from adaptive_amd.captions import Vocabulary, coco_results, dump_results, ids_to_sentences
from adaptive_amd.checkpoint import checkpoint_name, load_checkpoint, save_checkpoint, start_epoch


def _reference_loop(ids, vocab):
    """utils.py:176-190 verbatim in behaviour: per row, stop before the first <end>."""
    out = []
    for row in ids:
        words = []
        for word_id in row:
            word = vocab.idx2word[word_id]
            if word == "<end>":
                break
            words.append(word)
        out.append(" ".join(words))
    return out


def _vocab(n=40):
    return Vocabulary.with_specials(f"w{i}" for i in range(n))


def test_vocabulary_semantics():
    v = _vocab(3)
    assert [v.idx2word[i] for i in range(4)] == ["<pad>", "<start>", "<end>", "<unk>"]
    assert len(v) == 7 and v("w2") == 6 and v("nope") == v("<unk>") == 3
    v.add_word("w0")  # duplicates are ignored
    assert len(v) == 7


def test_ids_to_sentences_matches_reference_loop():
    v = _vocab()
    rng = np.random.default_rng(0)
    ids = rng.integers(0, len(v), size=(257, 20))
    ids[5, :] = 2          # <end> first: empty caption
    ids[6, :] = 7          # no <end>: all T words
    ids[7, 19] = 2
    assert ids_to_sentences(torch.from_numpy(ids), v) == _reference_loop(ids, v)
    assert ids_to_sentences(ids, v)[5] == ""


def test_unknown_id_raises_only_before_end():
    v = _vocab(4)
    ok = np.array([[5, 2, 999]])       # the bad id sits after <end>: never looked up
    assert ids_to_sentences(ok, v) == _reference_loop(ok, v) == ["w1"]
    with pytest.raises(KeyError):
        ids_to_sentences(np.array([[5, 999, 2]]), v)


def test_vocab_json_round_trip_and_results(tmp_path):
    v = _vocab(10)
    v.to_json(tmp_path / "vocab.json")
    w = Vocabulary.from_json(tmp_path / "vocab.json")
    assert w.idx2word == v.idx2word and w.word2idx == v.word2idx and w.idx == v.idx
    res = coco_results(np.array([[5, 6, 2, 0], [4, 4, 4, 4]]), [42, 7], w)
    assert res == [{"image_id": 42, "caption": "w1 w2"}, {"image_id": 7, "caption": "w0 w0 w0 w0"}]
    dump_results(res, tmp_path / "r.json")
    assert json.load(open(tmp_path / "r.json")) == res
    with pytest.raises(ValueError):
        coco_results(np.zeros((2, 3), np.int64), [1], w)


def test_checkpoint_round_trip_reference_names(tmp_path):
    m = Encoder2Decoder(Config()).load_synthetic(5)
    path = save_checkpoint(m, str(tmp_path), 0.987654, 12)
    assert path.endswith(checkpoint_name(0.987654, 12)) and path.endswith("cider-0.9877_model-12.pkl")
    sd = torch.load(path, weights_only=True)
    assert list(sd) == list(m.state_dict())
    sd["encoder.resnet_conv.0.weight"] = torch.zeros(3)   # a reference checkpoint carries the trunk
    torch.save(sd, tmp_path / "ref.pkl")
    m2 = Encoder2Decoder(Config())
    load_checkpoint(m2, str(tmp_path / "ref.pkl"))
    for (k, a), b in zip(m.state_dict().items(), m2.state_dict().values()):
        assert torch.equal(a, b), k


def test_start_epoch_parsing_matches_reference():
    assert start_epoch("models/adaptive-7.pkl") == 8
    assert start_epoch("/x/y/cider-1.0312_model-12.pkl") == 2   # the reference's own quirk


def test_checkpoint_with_trunk_loads_strictly_in_reference_shaped_module(tmp_path):
    """A trunk-less model's file plus a torchvision-layout trunk state (save_checkpoint(...,
    trunk_state=)) is complete: a reference-shaped module (the trunk included, as
    model_factory.py:16 builds it) loads it with strict=True; without trunk_state it does not."""
    from adaptive_amd.trunk import resnet_conv
    m = Encoder2Decoder(Config()).load_synthetic(5)
    trunk = resnet_conv()
    full = save_checkpoint(m, str(tmp_path), 0.5, 1, trunk_state=trunk.state_dict())
    ref_shaped = Encoder2Decoder(Config(), trunk=True)
    load_checkpoint(ref_shaped, full, strict=True)
    for k, v in m.state_dict().items():
        assert torch.equal(ref_shaped.state_dict()[k], v), k
    for k, v in trunk.state_dict().items():
        assert torch.equal(ref_shaped.state_dict()["encoder.resnet_conv." + k], v), k
    bare = save_checkpoint(m, str(tmp_path), 0.5, 2)
    with pytest.raises(RuntimeError, match="Missing key"):
        load_checkpoint(Encoder2Decoder(Config(), trunk=True), bare, strict=True)
    with pytest.raises(ValueError):
        save_checkpoint(ref_shaped, str(tmp_path), 0.5, 3, trunk_state=trunk.state_dict())
