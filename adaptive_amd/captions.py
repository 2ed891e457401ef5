"""Caption post-processing around the decode: token ids -> words -> the COCO
results JSON the reference's evaluation writes.

Mirrors ``code_src/data/build_vocab.py:9-28`` (``Vocabulary``) and the id->word loop of
``coco_eval`` (``code_src/tools/utils.py:176-193``): each row of the sampler's ids is read left
to right, words are looked up in ``idx2word``, the sentence stops before the first ``<end>`` and
is joined with single spaces.  The per-row cut is vectorised (one numpy pass over the [B, T] ids
finds every row's first ``<end>``), so post-processing a 512-caption batch costs microseconds
next to the decode instead of 10k Python iterations.

The reference stores its vocabulary as a pickle (``code_src/data/vocab.pkl``, loaded with
``pickle.load`` at ``utils.py:124``, ``train.py:38``).  Unpickling executes code from the file,
so this module reads and writes a plain JSON form instead; a maintainer converts an existing
``vocab.pkl`` once on the reference side (``Vocabulary.to_json``'s docstring shows how).
"""
from __future__ import annotations

import json
from typing import Dict, Iterable, List, Sequence

import numpy as np

PAD, START, END, UNK = "<pad>", "<start>", "<end>", "<unk>"


class Vocabulary:
    """``build_vocab.py:9-28``: ``word2idx`` / ``idx2word`` dicts, ``add_word``, ``__call__``
    (unknown words map to ``<unk>``) and ``__len__``, with the same attribute names so code that
    touches them directly keeps working."""

    def __init__(self):
        self.word2idx: Dict[str, int] = {}
        self.idx2word: Dict[int, str] = {}
        self.idx = 0

    def add_word(self, word: str) -> None:
        if word not in self.word2idx:
            self.word2idx[word] = self.idx
            self.idx2word[self.idx] = word
            self.idx += 1

    def __call__(self, word: str) -> int:
        if word not in self.word2idx:
            return self.word2idx[UNK]
        return self.word2idx[word]

    def __len__(self) -> int:
        return len(self.word2idx)

    @classmethod
    def with_specials(cls, words: Iterable[str] = ()) -> "Vocabulary":
        """The construction order of ``build_vocab.py:47-55``: ``<pad> <start> <end> <unk>`` get
        ids 0-3, then the corpus words in order."""
        v = cls()
        for w in (PAD, START, END, UNK):
            v.add_word(w)
        for w in words:
            v.add_word(w)
        return v

    # ------------------------------------------------------------------ JSON form
    def to_json(self, path: str) -> None:
        """Write ``{"idx2word": [...]}`` (ids are the list positions).

        Converting the reference's pickle, on the reference side where it is trusted::

            import pickle, json
            from code_src.data.build_vocab import Vocabulary
            v = pickle.load(open("code_src/data/vocab.pkl", "rb"))
            json.dump({"idx2word": [v.idx2word[i] for i in range(len(v))]}, open("vocab.json", "w"))
        """
        with open(path, "w") as f:
            json.dump({"idx2word": [self.idx2word[i] for i in range(self.idx)]}, f)

    @classmethod
    def from_json(cls, path: str) -> "Vocabulary":
        with open(path) as f:
            words = json.load(f)["idx2word"]
        v = cls()
        for w in words:
            if w in v.word2idx:
                raise ValueError(f"duplicate word {w!r} in {path}")
            v.add_word(w)
        return v

    def words_array(self) -> np.ndarray:
        """idx2word as an object array indexed by id (KeyError for a gap, as the dict lookup)."""
        return np.array([self.idx2word[i] for i in range(self.idx)], dtype=object)


def ids_to_sentences(ids, vocab: Vocabulary) -> List[str]:
    """``utils.py:176-190`` for a whole batch: ids ``[B, T]`` (torch tensor on any device, or
    array-like) -> B sentences, each the words before the row's first ``<end>``.  An id outside
    the vocabulary raises ``KeyError`` like ``vocab.idx2word[word_id]`` — but only for ids that
    precede the row's first ``<end>``: the reference loop stops at ``<end>`` before looking the
    rest up."""
    if hasattr(ids, "detach"):
        ids = ids.detach().cpu().numpy()
    ids = np.asarray(ids)
    if ids.ndim != 2:
        raise ValueError(f"ids must be [B, T], got shape {ids.shape}")
    B, T = ids.shape
    end = vocab.word2idx.get(END, None)
    if end is None or T == 0:
        cut = np.full(B, T, dtype=np.int64)
    else:
        hit = ids == end
        cut = np.where(hit.any(axis=1), hit.argmax(axis=1), T)
    words = vocab.words_array()
    n = len(words)
    out = []
    for b in range(B):
        row = ids[b, : cut[b]]
        if row.size and (row.min() < 0 or row.max() >= n):
            bad = int(row[(row < 0) | (row >= n)][0])
            raise KeyError(bad)
        out.append(" ".join(words[row]))
    return out


def coco_results(ids, img_ids: Sequence[int], vocab: Vocabulary) -> List[dict]:
    """``utils.py:192-193``: ``[{'image_id': int, 'caption': sentence}, ...]`` in batch order."""
    sentences = ids_to_sentences(ids, vocab)
    if len(img_ids) != len(sentences):
        raise ValueError(f"{len(img_ids)} image ids for {len(sentences)} captions")
    return [{"image_id": int(i), "caption": s} for i, s in zip(img_ids, sentences)]


def dump_results(results: List[dict], path: str) -> None:
    """``utils.py:221`` (``json.dump(results, open(resFile, 'w'))``)."""
    with open(path, "w") as f:
        json.dump(results, f)
