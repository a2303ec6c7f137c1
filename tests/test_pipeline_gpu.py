"""BASELINE.json configs[4] end to end on the GPU: an MLS-style stream (each utterance U[10, 20] s encoded alone,
``encode_audio_chunk`` semantics, ``mls-en-mimi-pretrain/process_shard.py:302-307``) and then codec-BPE training
over the emitted codes (``codec-bpe/train_bpe_recipe.txt:18-28`` -> ``bpe_trainer.py:107-166``).

Checks: the GPU merge loop over the engine's own codes gives the merges of (1) the CPU oracle of the merge loop
(``oracle/bpe_ref.py``) and (2) HF ``tokenizers`` 0.22.2 trained live on the ``codes_to_chars`` strings of the
same 30 s chunks, with the reference recipe's tokenizer setup (NFKC, Metaspace without prefix, max_token_length
= ngrams x codebooks + 1, as ``tests/golden/make_bpe_golden.py``).  ``codec_bpe`` itself is absent: its wrapper
module stays unpinned, the merge semantics are pinned to ``tokenizers``.
"""
import json

import numpy as np
import pytest
import torch

from mimi_hip import bpe, synthetic
from mimi_hip.codes import codes_to_chars
from mimi_hip.config import encoded_length
from oracle.bpe_ref import train_bpe

pytestmark = pytest.mark.gpu

NCB, CBS, FR, CHUNK_S = 8, 2048, 12.5, 30


def tokenizers_merges(strings, vocab_size, max_len):
    from tokenizers import Tokenizer, pre_tokenizers, trainers
    from tokenizers.models import BPE
    from tokenizers.normalizers import NFKC
    tok = Tokenizer(BPE(unk_token=None))
    tok.normalizer = NFKC()
    tok.pre_tokenizer = pre_tokenizers.Metaspace(replacement="▁", prepend_scheme="never")
    alphabet = [chr(i) for i in range(0xE000, 0xE000 + NCB * CBS)]
    tok.train_from_iterator(strings, trainer=trainers.BpeTrainer(
        vocab_size=vocab_size, min_frequency=2, special_tokens=["<pad>"], limit_alphabet=len(alphabet),
        initial_alphabet=alphabet, max_token_length=max_len, show_progress=False))
    j = json.loads(tok.to_str())
    vocab = j["model"]["vocab"]
    return [(vocab[a], vocab[b], vocab[a + b]) for a, b in (tuple(m) for m in j["model"]["merges"])]


@pytest.mark.parametrize("ngrams", [2, None])
def test_mls_stream_then_bpe(state_dict, ngrams):
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from mimi_hip.encoder import MimiEncoder
    from mimi_hip.model import MimiHipModel
    model = MimiHipModel(state_dict, device="cuda:0")
    enc = MimiEncoder(device="cuda:0", model=model, num_quantizers=NCB, concurrency=2)
    lengths = synthetic.random_lengths(10, 10.0, 20.0, seed=41)
    audio = [synthetic.speech_like(L, 41, i) for i, L in enumerate(lengths)]
    audio += audio[:4]  # repeated utterances (re-reads in a shard list): every pair of theirs occurs twice
    codes = enc.encode_audio_chunks(audio, 24000)
    for a, c in zip(audio, codes):
        assert c.shape == (NCB, encoded_length(len(a))) and c.dtype == np.int64
    for i in range(4):
        assert np.array_equal(codes[10 + i], codes[i])

    vocab_size = NCB * CBS + 1 + 400
    tr = bpe.Trainer(NCB, CBS, codec_framerate=FR, chunk_size_secs=CHUNK_S, vocab_size=vocab_size, min_frequency=2,
                     pad_token="<pad>", max_token_codebook_ngrams=ngrams)
    tok = tr.train_codes([c.copy() for c in codes])
    got_tokens, got_merges = tr.last_tokens, tr.last_merges
    assert len(got_merges) > 0

    # (1) CPU oracle of the merge loop on the same words
    words, counts = tr.words([c.copy() for c in codes])
    ml = tr._max_token_length()
    toks, merges = train_bpe([w + 1 for w in words], counts, NCB * CBS, 1, vocab_size, 2,
                             ml + 1 if ml is not None else None)
    assert got_merges == merges
    assert got_tokens == [t for t in toks[1 + NCB * CBS:]]

    # (2) tokenizers on the reference's chunk strings (bpe_trainer.py:73-105: 30 s chunks -> codes_to_chars)
    step = int(CHUNK_S * FR)
    strings = [codes_to_chars(c[:, i:i + step].copy(), CBS) for c in codes for i in range(0, c.shape[1], step)]
    ref = tokenizers_merges(strings, vocab_size, ml + 1 if ml is not None else None)
    ids = {t: i for i, t in enumerate(toks) if i >= 1}
    mine = [(a, b, ids[toks[a] + toks[b]]) for a, b in merges]
    assert mine == ref
    assert len(tok.get_vocab()) == 1 + NCB * CBS + len(got_tokens)
