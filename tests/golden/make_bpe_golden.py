"""Codec-BPE fixtures (run in the survey container only; outputs are committed).

    python tests/golden/make_bpe_golden.py

The reference recipe (``/root/reference/codec-bpe/train_bpe_recipe.txt:18-28``; ``bpe_trainer.py:107-166``)
trains ``codec_bpe``'s SentencePieceBPETokenizer -- HF ``tokenizers`` 0.22.2 with an NFKC normalizer, a
Metaspace pre-tokenizer (no prefix space) and ``BpeTrainer(max_token_length=...)`` -- on ``codes_to_chars``
strings of 30 s chunks.  ``codec_bpe`` is not installed; its tokenizer class is restated from ``tokenizers``'
own ``implementations/sentencepiece_bpe.py`` with ``max_token_length`` forwarded (what ``bpe_trainer.py:147-156``
calls), and its ``codes_to_chars`` as the reference's ``librispeech-mimi/utils.py:18-37`` (same formula; the
codec_bpe module itself is unpinned).  Fixture: a synthetic code corpus (a seeded Markov source with repeated
"silence" frames, Zipf-like codes, so codebook 3 hits the NFKC-rewritten characters U+F900-U+FFEF), the chunk
strings, and the trained merges as (left id, right id, new id) of ``tokenizers`` itself, for two settings:
the recipe's (``max_token_codebook_ngrams`` 2 -> ``max_token_length`` 17) and unlimited length.
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from make_golden import OUT, REF, load_reference_module, stub_module  # noqa: E402

NCB, CBS, FR = 8, 2048, 12.5
CHUNK = int(30 * FR)


def corpus(seed=5, n_utt=24):
    rng = np.random.default_rng(seed)
    zipf = 1.0 / np.arange(1, CBS + 1) ** 1.1
    zipf /= zipf.sum()
    perm = np.stack([rng.permutation(CBS) for _ in range(NCB)])
    silence = perm[:, 0]
    utts = []
    for u in range(n_utt):
        T = int(rng.integers(60, 900))
        codes = np.empty((NCB, T), np.int64)
        for t in range(T):
            r = rng.random()
            if r < 0.15:
                codes[:, t] = silence
            elif r < 0.35 and t > 0:
                codes[:, t] = codes[:, t - 1]
                k = rng.integers(0, NCB)
                codes[k:, t] = perm[np.arange(k, NCB), rng.choice(CBS, NCB - k, p=zipf)]
            else:
                codes[:, t] = perm[np.arange(NCB), rng.choice(CBS, NCB, p=zipf)]
        utts.append(codes)
    return utts


def train_reference(strings, vocab_size, max_len, specials=("<pad>",)):
    from tokenizers import Tokenizer, decoders, pre_tokenizers, trainers
    from tokenizers.models import BPE
    from tokenizers.normalizers import NFKC
    tok = Tokenizer(BPE(unk_token=None))
    tok.normalizer = NFKC()
    tok.pre_tokenizer = pre_tokenizers.Metaspace(replacement="▁", prepend_scheme="never")
    tok.decoder = decoders.Metaspace(replacement="▁", prepend_scheme="never")
    alphabet = [chr(i) for i in range(0xE000, 0xE000 + NCB * CBS)]
    tr = trainers.BpeTrainer(vocab_size=vocab_size, min_frequency=2, special_tokens=list(specials),
                             limit_alphabet=len(alphabet), initial_alphabet=alphabet, max_token_length=max_len,
                             show_progress=False)
    tok.train_from_iterator(strings, trainer=tr)
    return json.loads(tok.to_str())


def main():
    from transformers import MimiModel  # noqa: F401  (before the librosa stub, as make_golden.py does)
    stub_module("librosa")
    utils_mod = load_reference_module(os.path.join(REF, "librispeech-mimi", "utils.py"), "ref_utils")
    utts = corpus()
    strings = []
    for codes in utts:
        for i in range(0, codes.shape[1], CHUNK):
            strings.append(utils_mod.codes_to_chars(codes[:, i:i + CHUNK].copy(), codebook_size=CBS))
    arrays = {f"utt{i}": u.astype(np.int16) for i, u in enumerate(utts)}
    meta = {"num_codebooks": NCB, "codebook_size": CBS, "codec_framerate": FR, "chunk_size_secs": 30,
            "unicode_offset": 0xE000, "special_tokens": ["<pad>"], "min_frequency": 2, "n_utterances": len(utts),
            "n_chunks": len(strings), "tokenizers": __import__("tokenizers").__version__, "cases": {}}
    for name, vocab_size, ngrams in (("recipe", NCB * CBS + 1 + 2500, 2), ("unlimited", NCB * CBS + 1 + 1500, None)):
        max_len = None if ngrams is None else ngrams * NCB + 1  # bpe_trainer.py:133-135, 146-148
        j = train_reference(strings, vocab_size, max_len)
        vocab = j["model"]["vocab"]
        merges = [tuple(m) for m in j["model"]["merges"]]
        arrays[f"{name}_merges"] = np.array([(vocab[a], vocab[b], vocab[a + b]) for a, b in merges], np.int32)
        meta["cases"][name] = {"vocab_size": vocab_size, "max_token_codebook_ngrams": ngrams,
                               "n_merges": len(merges), "final_vocab": len(vocab)}
        print(name, "merges", len(merges), "vocab", len(vocab))
    np.savez_compressed(os.path.join(OUT, "bpe.npz"), **arrays)
    with open(os.path.join(OUT, "bpe_meta.json"), "w") as f:
        json.dump(meta, f, indent=1)


if __name__ == "__main__":
    main()
