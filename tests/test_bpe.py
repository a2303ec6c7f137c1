"""Codec-BPE over emitted codes: the host corpus pipeline, the CPU oracle of the merge
loop, and the GPU trainer, against HF ``tokenizers`` 0.22.2 (fixtures of tests/golden/make_bpe_golden.py, and
live re-training where ``tokenizers`` is importable)."""
import json
import os
import random

import numpy as np
import pytest

from mimi_hip import bpe
from mimi_hip.codes import codes_to_codepoints
from oracle.bpe_ref import train_bpe

HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def fixture():
    with open(os.path.join(HERE, "bpe_meta.json")) as f:
        meta = json.load(f)
    with np.load(os.path.join(HERE, "bpe.npz"), allow_pickle=False) as z:
        arrays = {k: z[k] for k in z.files}
    utts = [arrays[f"utt{i}"].astype(np.int64) for i in range(meta["n_utterances"])]
    return meta, utts, arrays


def trainer_for(meta, case):
    c = meta["cases"][case]
    return bpe.Trainer(meta["num_codebooks"], meta["codebook_size"], codec_framerate=meta["codec_framerate"],
                       chunk_size_secs=meta["chunk_size_secs"], vocab_size=c["vocab_size"],
                       min_frequency=meta["min_frequency"], pad_token="<pad>",
                       max_token_codebook_ngrams=c["max_token_codebook_ngrams"], unicode_offset=meta["unicode_offset"])


def merges_from_oracle(tr, utts):
    words, counts = tr.words([u.copy() for u in utts])
    n_base = tr.num_codebooks * tr.codebook_size
    n_sp = len(tr.special_tokens)
    ml = tr._max_token_length()
    tokens, merges = train_bpe([w + n_sp for w in words], counts, n_base, n_sp, tr.vocab_size, tr.min_frequency,
                               ml + 1 if ml is not None else None)
    ids = {t: i for i, t in enumerate(tokens) if i >= n_sp}
    return np.array([(a, b, ids[tokens[a] + tokens[b]]) for a, b in merges], np.int32).reshape(-1, 3)


@pytest.mark.parametrize("case", ["recipe", "unlimited"])
def test_oracle_reproduces_tokenizers_fixture(case):
    """Host pipeline (codes -> NFKC-model words) + oracle merge loop == tokenizers' merges, in order."""
    meta, utts, arrays = fixture()
    got = merges_from_oracle(trainer_for(meta, case), utts)
    ref = arrays[f"{case}_merges"]
    assert got.shape == ref.shape and np.array_equal(got, ref)


def test_char_model_matches_tokenizers_pretokenization():
    """The code-character model (drops, splits, canonical reordering) gives exactly the words tokenizers trains on
    (its NFKC normalizer + Metaspace pre-tokenizer + alphabet filter), on sequences dense in the rewritten and
    combining characters."""
    tokenizers = pytest.importorskip("tokenizers")
    from tokenizers import pre_tokenizers
    from tokenizers.normalizers import NFKC
    first, count = 0xE000, 8 * 2048
    m = bpe.CharModel(first, count)
    nrm, pt = NFKC(), pre_tokenizers.Metaspace(replacement="▁", prepend_scheme="never")
    special = np.nonzero(m.cls != bpe.KEEP_STARTER)[0]
    by_cb = [special[(special // 2048) == k] - 2048 * k for k in range(8)]
    rng = random.Random(0)
    for _ in range(3000):
        T = rng.randint(0, 30)
        codes = np.array([[by_cb[k][rng.randrange(len(by_cb[k]))] if len(by_cb[k]) and rng.random() < 0.6
                           else rng.randrange(2048) for _ in range(T)] for k in range(8)], dtype=np.int64).reshape(8, T)
        cps = codes_to_codepoints(codes, 2048)
        s = "".join(map(chr, cps))
        ref = [[ord(c) - first for c in p if first <= ord(c) < first + count] for p, _ in
               pt.pre_tokenize_str(nrm.normalize_str(s))]
        assert [w for w in ref if w] == [list(w) for w in m.words(cps) if len(w)], tokenizers.__version__


def test_oracle_matches_live_tokenizers_on_random_corpora():
    tokenizers = pytest.importorskip("tokenizers")
    from tokenizers import Tokenizer, pre_tokenizers, trainers
    from tokenizers.models import BPE
    rng = random.Random(3)
    for case in range(80):
        nalpha = rng.randint(2, 8)
        alphabet = [chr(0xE000 + i) for i in range(nalpha)]
        seqs = ["".join(rng.choice(alphabet[:rng.randint(1, nalpha)]) for _ in range(rng.randint(0, 50)))
                for _ in range(rng.randint(1, 40))]
        ml = [None, 2, 3, 4, 5, 8][case % 6]
        mf = [1, 2, 3][case % 3]
        vs = 1 + nalpha + rng.randint(0, 60)
        tok = Tokenizer(BPE(unk_token=None))
        tok.pre_tokenizer = pre_tokenizers.Metaspace(replacement="▁", prepend_scheme="never")
        tok.train_from_iterator(seqs, trainer=trainers.BpeTrainer(
            vocab_size=vs, min_frequency=mf, special_tokens=["<pad>"], limit_alphabet=nalpha,
            initial_alphabet=alphabet, max_token_length=ml, show_progress=False))
        j = json.loads(tok.to_str())
        words = {}
        for s in seqs:
            words[s] = words.get(s, 0) + 1
        toks, merges = train_bpe([[1 + ord(c) - 0xE000 for c in w] for w in words], list(words.values()), nalpha, 1,
                                 vs, mf, ml)
        spell = lambda t: "".join(chr(0xE000 + i) for i in toks[t])  # noqa: E731
        assert [tuple(m) for m in j["model"]["merges"]] == [(spell(a), spell(b)) for a, b in merges], \
            (case, tokenizers.__version__)


def test_trainer_argument_checks():
    with pytest.raises(ValueError, match="codec_framerate must also be set"):
        bpe.Trainer(8, 2048, chunk_size_secs=30, vocab_size=20000, pad_token="<pad>")
    with pytest.raises(ValueError, match="Either pad_token or eos_token"):
        bpe.Trainer(8, 2048, vocab_size=20000)
    with pytest.raises(ValueError, match="must be at least 16385"):
        bpe.Trainer(8, 2048, vocab_size=16000, pad_token="<pad>")
    with pytest.raises(ValueError, match="non-negative"):
        bpe.Trainer(8, 2048, vocab_size=20000, pad_token="<pad>", max_token_codebook_ngrams=-1)
    t = bpe.Trainer(8, 2048, vocab_size=20000, eos_token="</s>", pad_token="<pad>", special_tokens=["<audio>"])
    assert t.special_tokens == ["<pad>", "</s>", "<audio>"]  # inserted at the front, as bpe_trainer.py:57-60


def test_codes_dtype_quirk_matches_reference():
    """The reference adds the offsets in the codes' dtype (codes_to_chars(copy_before_conversion=False)): uint16
    codes of 8 codebooks overflow (numpy >= 2 raises), int64 codes do not."""
    u16 = np.zeros((8, 4), np.uint16)
    with pytest.raises(OverflowError):
        codes_to_codepoints(u16, 2048, copy_before_conversion=False)
    assert codes_to_codepoints(u16.astype(np.int64), 2048)[7] == 0xE000 + 7 * 2048


@pytest.mark.gpu
@pytest.mark.parametrize("case", ["recipe", "unlimited"])
def test_gpu_trainer_reproduces_tokenizers_fixture(case, tmp_path):
    """The GPU merge loop through Trainer.train on .npy code files == tokenizers' merges; the assembled tokenizer
    encodes a chunk to the same ids as the reference-built one would (its vocab/merges are the fixture's)."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    meta, utts, arrays = fixture()
    # the reference's input format: an object array of per-utterance [8, T] code arrays per file
    for f in range(2):
        part = np.empty(len(utts[f::2]), dtype=object)
        for i, u in enumerate(utts[f::2]):
            part[i] = u
        np.save(tmp_path / f"codes_{f}.npy", part, allow_pickle=True)
    order = [u for f in range(2) for u in utts[f::2]]
    tr = trainer_for(meta, case)
    tok = tr.train(str(tmp_path))
    words, counts = tr.words([u.copy() for u in order])
    n_sp = len(tr.special_tokens)
    ml = tr._max_token_length()
    tokens, merges = bpe.train_words_gpu(words, counts, tr.num_codebooks * tr.codebook_size, n_sp, tr.vocab_size,
                                         tr.min_frequency, ml + 1 if ml is not None else None)
    spell = {t: n_sp + tr.num_codebooks * tr.codebook_size + i for i, t in enumerate(tokens)}
    base = lambda x: (x - n_sp,) if x < n_sp + tr.num_codebooks * tr.codebook_size else tokens[  # noqa: E731
        x - n_sp - tr.num_codebooks * tr.codebook_size]
    got = np.array([(a, b, spell[base(a) + base(b)]) for a, b in merges], np.int32).reshape(-1, 3)
    assert np.array_equal(got, arrays[f"{case}_merges"])
    vocab = tok.get_vocab()
    assert len(vocab) == meta["cases"][case]["final_vocab"]
    print(case, tr.last_stats)


@pytest.mark.gpu
def test_gpu_trainer_matches_oracle_on_random_corpora():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    rng = np.random.default_rng(11)
    for case in range(12):
        nalpha = int(rng.integers(2, 12))
        words = [rng.integers(0, max(1, int(rng.integers(1, nalpha + 1))), size=int(rng.integers(0, 60))).astype(np.int32)
                 for _ in range(int(rng.integers(1, 50)))]
        counts = rng.integers(1, 4, size=len(words))
        ml = [None, 2, 3, 5, 9][case % 5]
        vs = 1 + nalpha + int(rng.integers(0, 80))
        mf = 1 + case % 3
        toks, merges = train_bpe([w + 1 for w in words], counts, nalpha, 1, vs, mf, ml)
        gt, gm = bpe.train_words_gpu(words, counts, nalpha, 1, vs, mf, ml)
        assert gm == merges, case
        assert gt == [t for t in toks[1 + nalpha:]], case


@pytest.mark.gpu
def test_gpu_trainer_counts_beyond_2_30():
    """Pair counts are int64 on the device (two-sweep best pair): word counts near 2^31 push pair totals past 2^30
    and 2^32, where the old packed 64-bit max (count << 34) refused the corpus; merges == the oracle's."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    rng = np.random.default_rng(12)
    for case in range(4):
        nalpha = 6
        words = [rng.integers(0, nalpha, size=int(rng.integers(2, 20))).astype(np.int32) for _ in range(12)]
        counts = rng.integers((1 << 31) - 1000, (1 << 31) - 1, size=len(words))
        counts[case] = 3  # one rare word: its pairs lose every count tie
        toks, merges = train_bpe([w + 1 for w in words], counts, nalpha, 1, 1 + nalpha + 30, 2, None)
        gt, gm = bpe.train_words_gpu(words, counts, nalpha, 1, 1 + nalpha + 30, 2, None)
        assert gm == merges, case
        assert gt == [t for t in toks[1 + nalpha:]], case
