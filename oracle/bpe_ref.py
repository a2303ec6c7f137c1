"""ORACLE — test infrastructure only, never shipped, never on the product path.

CPU restatement of the BPE training step of the reference's codec-BPE recipe: ``Trainer.train``
(``/root/reference/codec-bpe/bpe_trainer.py:107-166``) hands the code strings to codec_bpe's
``SentencePieceBPETokenizer.train_from_iterator``, i.e. HF ``tokenizers`` 0.22.2 ``BpeTrainer`` (third-party Rust,
``tokenizers/src/models/bpe/trainer.rs``; not under /root/reference, and ``codec_bpe`` itself is not installed).
Restated from that trainer's published algorithm and pinned against ``tokenizers`` 0.22.2 itself
(``tests/golden/make_bpe_golden.py``; ``tests/test_bpe.py`` also re-trains live with ``tokenizers``):

* vocabulary = special tokens, then the alphabet sorted by code point, then one token per merge;
* pair counts over words weighted by word count; each step merges the pair of highest count, ties to the
  smallest (left id, right id); stop below ``min_frequency`` or at ``vocab_size``;
* a merge rewrites every word left to right (``aaa`` -> ``[aa] a``) and adjusts the counts of the pairs
  around each occurrence; a pair formed by a merge is counted only if its merged length is below
  ``max_token_length`` (the initial single-character pairs always are) -- which is why codec_bpe passes
  ``max_token_codebook_ngrams * num_codebooks + 1``;
* a merged string that is already a token reuses that token's id.
"""
from __future__ import annotations

import heapq
from typing import Dict, List, Optional, Sequence, Tuple


def train_bpe(words: Sequence[Sequence[int]], counts: Sequence[int], n_base: int, n_special: int, vocab_size: int,
              min_frequency: int = 2, max_token_length: Optional[int] = None, trace: Optional[list] = None
              ) -> Tuple[List[Tuple[int, ...]], List[Tuple[int, int]]]:
    """words: symbol ids (ids n_special .. n_special + n_base - 1 are the alphabet, in code point order).
    Returns (tokens, merges): tokens[i] = the alphabet indices (0-based) spelling token i >= n_special;
    merges = (left id, right id) in merge order."""
    tokens: List[Tuple[int, ...]] = [()] * n_special + [(i,) for i in range(n_base)]
    tok_id: Dict[Tuple[int, ...], int] = {t: i for i, t in enumerate(tokens) if i >= n_special}
    words = [list(w) for w in words]
    counts = list(counts)

    def elig(x, y):
        lx, ly = len(tokens[x]), len(tokens[y])
        return max_token_length is None or (lx == 1 and ly == 1) or lx + ly < max_token_length

    pc: Dict[Tuple[int, int], int] = {}
    where: Dict[Tuple[int, int], set] = {}
    for wi, w in enumerate(words):
        for x, y in zip(w, w[1:]):
            pc[(x, y)] = pc.get((x, y), 0) + counts[wi]
            where.setdefault((x, y), set()).add(wi)
    heap = [(-c, p) for p, c in pc.items() if c > 0]
    heapq.heapify(heap)
    merges: List[Tuple[int, int]] = []
    while len(tokens) < vocab_size and heap:
        negc, pair = heapq.heappop(heap)
        cur = pc.get(pair, 0)
        if -negc != cur:
            if cur > 0:
                heapq.heappush(heap, (-cur, pair))
            continue
        if cur < min_frequency or cur < 1:
            break
        a, b = pair
        new = tokens[a] + tokens[b]
        nid = tok_id.get(new)
        if nid is None:
            nid = len(tokens)
            tokens.append(new)
            tok_id[new] = nid
        merges.append(pair)
        if trace is not None:
            trace.append((cur, dict(pc)) if len(trace) < 3 else cur)
        touched = {}
        for wi in sorted(where.get(pair, ())):
            w = words[wi]
            c = counts[wi]
            i = 0
            out = []
            while i < len(w):
                if i + 1 < len(w) and w[i] == a and w[i + 1] == b:
                    # changes around this occurrence, as the word is rewritten left to right
                    if out:
                        left = out[-1]
                        pc[(left, a)] = pc.get((left, a), 0) - c
                        if elig(left, nid):
                            pc[(left, nid)] = pc.get((left, nid), 0) + c
                            touched.setdefault((left, nid), set()).add(wi)
                    if i + 2 < len(w):
                        right = w[i + 2]
                        pc[(b, right)] = pc.get((b, right), 0) - c
                        if elig(nid, right):
                            pc[(nid, right)] = pc.get((nid, right), 0) + c
                            touched.setdefault((nid, right), set()).add(wi)
                    out.append(nid)
                    i += 2
                else:
                    out.append(w[i])
                    i += 1
            words[wi] = out
        pc[pair] = 0
        for p, ws in touched.items():
            where.setdefault(p, set()).update(ws)
            if pc.get(p, 0) > 0:
                heapq.heappush(heap, (-pc[p], p))
    return tokens, merges
