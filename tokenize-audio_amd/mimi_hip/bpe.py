"""Codec-BPE training over emitted Mimi codes, with the merge loop on the GPU.

Mirrors the reference recipe's trainer (``/root/reference/codec-bpe/bpe_trainer.py``, which replaces codec_bpe's
``core/trainer.py``; run as ``python -m codec_bpe.train_tokenizer`` in ``codec-bpe/train_bpe_recipe.txt:18-28``):

* ``Trainer(num_codebooks, codebook_size, codec_framerate, chunk_size_secs, vocab_size, min_frequency,
  special_tokens, bos/eos/unk/pad_token, max_token_codebook_ngrams, unicode_offset)`` -- same arguments, checks
  and error messages (``bpe_trainer.py:12-71``);
* ``train(codes_path, codes_filter, num_files)`` -- ``.npy`` code files (one array, or an object array of
  per-utterance ``[num_codebooks, T]`` arrays), cut into ``chunk_size_secs`` chunks, each chunk one
  training sequence of ``codes_to_chars`` characters (``bpe_trainer.py:73-105``), base alphabet = all
  ``num_codebooks * codebook_size`` code characters, tokens at most ``max_token_codebook_ngrams *
  num_codebooks`` characters (``:107-166``).

The reference trains through HF ``tokenizers`` (codec_bpe's ``SentencePieceBPETokenizer``: NFKC normalizer,
Metaspace pre-tokenizer, ``BpeTrainer``).  Here:

1. host (numpy): codes -> code points per chunk -> the normalizer's effect on them -> words.  The code
   characters run into Unicode blocks that NFKC rewrites (codebook 3 at offset 0xE000 covers U+F800-U+FFFF:
   1,539 characters change, 21 into text containing a space, where the pre-tokenizer splits the chunk) and
   into combining marks that NFKC reorders.  ``data/bpe_unicode.json`` records what ``tokenizers`` does with
   every such character (``tools/make_bpe_unicode.py``); per chunk: characters NFKC replaces are dropped (their
   replacements are never code characters, so the trainer's alphabet filter drops them), those whose
   replacement holds a space split the word, and the surviving combining marks are stably sorted by combining
   class inside each run between starters -- exactly the words ``tokenizers`` trains on
   (``tests/test_bpe.py`` checks it against ``tokenizers`` itself);
2. GPU (``bpe.hip`` through ``mimi_bpe_*``): pair counts in a device hash table, one merge per step applied to
   every word in parallel (left-to-right occurrence rule, count deltas), best pair by a packed 64-bit max
   (count, then smallest pair) -- the ``BpeTrainer`` rules restated in ``oracle/bpe_ref.py``;
3. the trained vocabulary and merges are assembled into the same ``tokenizers`` BPE tokenizer (NFKC,
   Metaspace) and, when ``transformers`` is importable, a ``PreTrainedTokenizerFast`` as the reference returns.

One quirk is kept rather than fixed: the reference adds the offsets in the codes' own dtype
(``codes_to_chars(..., copy_before_conversion=False)``); on uint16 files with 8 codebooks that overflows
(numpy >= 2 raises OverflowError, numpy 1.x wraps codebooks 4-7 to U+0000-U+1FFF).  ``codes_to_codepoints``
does the same add, so the same inputs fail or wrap the same way.
"""
from __future__ import annotations

import ctypes
import glob
import json
import os
import time
import warnings
from typing import Dict, Iterable, List, Optional, Sequence, Tuple, Union

import numpy as np

from .codes import UNICODE_OFFSET, codes_to_codepoints

_DATA = os.path.join(os.path.dirname(os.path.abspath(__file__)), "data", "bpe_unicode.json")

# character classes of the normalizer model
KEEP_STARTER, KEEP_MARK, DROP_STARTER, DROP_MARK, SPLIT = 0, 1, 2, 3, 4


def validate_unicode_offset(unicode_offset: int, num_codebooks: int, codebook_size: int) -> int:
    end = unicode_offset + num_codebooks * codebook_size
    if unicode_offset < 0 or end > 0x110000 or (unicode_offset < 0xE000 and end > 0xD800):
        raise ValueError(f"unicode_offset {unicode_offset:#x} puts the {num_codebooks} x {codebook_size} code "
                         f"characters outside valid code points")
    return unicode_offset


_unicode = None


def _unicode_data():
    global _unicode
    if _unicode is None:
        with open(_DATA) as f:
            d = json.load(f)
        _unicode = ({int(k): v for k, v in d["nfkc"].items()}, {int(k): v for k, v in d["ccc"].items()})
    return _unicode


class CharModel:
    """Class and combining class of each code character under tokenizers' NFKC (see module docstring)."""

    def __init__(self, first: int, count: int):
        nfkc, ccc = _unicode_data()
        self.first, self.count = first, count
        self.cls = np.zeros(count, np.uint8)
        self.ccc = np.zeros(count, np.uint8)
        for cp in range(first, first + count):
            out = nfkc.get(cp)
            i = cp - first
            if out is None:
                c = ccc.get(cp, 0)
                self.ccc[i] = c
                self.cls[i] = KEEP_MARK if c else KEEP_STARTER
                continue
            if any(first <= o < first + count for o in out):
                raise NotImplementedError(f"NFKC maps code character {cp:#x} onto another code character")
            if 0x20 in out:
                self.cls[i] = SPLIT
            elif any(ccc.get(o, 0) == 0 for o in out):
                self.cls[i] = DROP_STARTER
            else:
                self.cls[i] = DROP_MARK

    def words(self, cps: np.ndarray) -> List[np.ndarray]:
        """Code points of one training sequence -> the alphabet indices of each of its words (tokenizers'
        NFKC + Metaspace split + alphabet filter)."""
        idx = cps.astype(np.int64) - self.first
        if idx.size == 0:
            return [idx]
        if idx.min() < 0 or idx.max() >= self.count:
            raise ValueError("code characters outside the trainer's alphabet")
        cls = self.cls[idx]
        marks = np.nonzero(cls == KEEP_MARK)[0]
        if marks.size > 1:
            # canonical ordering: stable sort of the kept marks by combining class inside each run of
            # non-starters (dropped marks take part in the run but do not survive, so they cannot reorder)
            starter = (cls == KEEP_STARTER) | (cls == DROP_STARTER) | (cls == SPLIT)
            run = np.cumsum(starter)[marks]
            key = run.astype(np.int64) * 256 + self.ccc[idx[marks]]
            order = np.argsort(key, kind="stable")
            if (order != np.arange(order.size)).any():
                idx = idx.copy()
                idx[marks] = idx[marks[order]]
        keep = (cls == KEEP_STARTER) | (cls == KEEP_MARK)
        splits = np.nonzero(cls == SPLIT)[0]
        if splits.size == 0:
            return [idx[keep]]
        out, start = [], 0
        for s in splits:
            seg = slice(start, s)
            out.append(idx[seg][keep[seg]])
            start = s + 1
        out.append(idx[start:][keep[start:]])
        return out


def get_codes_files(codes_path: str, codes_filter: Optional[Union[str, List[str]]] = None,
                    num_files: Optional[int] = None) -> List[str]:
    """``.npy`` files under codes_path (sorted); codes_filter keeps paths containing (any of) the filter
    string(s); num_files keeps the first n."""
    files = sorted(glob.glob(os.path.join(codes_path, "**", "*.npy"), recursive=True))
    if codes_filter:
        flt = [codes_filter] if isinstance(codes_filter, str) else list(codes_filter)
        files = [f for f in files if any(x in f for x in flt)]
    if num_files is not None:
        files = files[:num_files]
    if not files:
        raise ValueError(f"no codes files found in {codes_path}")
    return files


def _utterances(codes_file: str) -> List[np.ndarray]:
    codes_data = np.load(codes_file, allow_pickle=True)  # the reference's loader (object arrays of utterances)
    if isinstance(codes_data, np.ndarray) and codes_data.dtype == object and len(codes_data.shape) == 0:
        codes_list = codes_data.item()
        if not isinstance(codes_list, list):
            codes_list = [codes_list]
    elif isinstance(codes_data, np.ndarray) and codes_data.dtype == object and len(codes_data.shape) == 1:
        codes_list = list(codes_data)
    else:
        codes_list = [codes_data]
    return codes_list


class Trainer:
    def __init__(self, num_codebooks: int, codebook_size: int, codec_framerate: Optional[float] = None,
                 chunk_size_secs: Optional[int] = None, vocab_size: int = 30000, min_frequency: int = 2,
                 special_tokens: Optional[List[str]] = None, bos_token: Optional[str] = None,
                 eos_token: Optional[str] = None, unk_token: Optional[str] = None, pad_token: Optional[str] = None,
                 max_token_codebook_ngrams: Optional[int] = None, unicode_offset: int = UNICODE_OFFSET,
                 device: Union[int, str] = 0):
        if chunk_size_secs is not None:
            if codec_framerate is None:
                raise ValueError("If chunk_size_secs is set, codec_framerate must also be set.")
            if chunk_size_secs < 1:
                raise ValueError("chunk_size_secs must be a positive integer >= 1.")
        if eos_token is None and pad_token is None:
            raise ValueError(
                "Either pad_token or eos_token should be set, otherwise padded batching will not work with this "
                "tokenizer.")
        if max_token_codebook_ngrams is not None and max_token_codebook_ngrams < 0:
            raise ValueError("max_token_codebook_ngrams must be a non-negative integer (0 or greater).")
        self.num_codebooks = num_codebooks
        self.codebook_size = codebook_size
        self.codec_framerate = codec_framerate
        self.chunk_size_secs = chunk_size_secs
        self.vocab_size = vocab_size
        self.min_frequency = min_frequency
        self.special_tokens = list(special_tokens) if special_tokens is not None else []
        self.bos_token, self.eos_token, self.unk_token, self.pad_token = bos_token, eos_token, unk_token, pad_token
        self.max_token_codebook_ngrams = max_token_codebook_ngrams
        self.unicode_offset = validate_unicode_offset(unicode_offset, num_codebooks, codebook_size)
        self.device = device if isinstance(device, int) else int(str(device).split(":")[-1] or 0)
        for special_token in [self.eos_token, self.bos_token, self.unk_token, self.pad_token]:
            if special_token is not None and special_token not in self.special_tokens:
                self.special_tokens.insert(0, special_token)
        min_vocab_size = self.num_codebooks * self.codebook_size + len(self.special_tokens)
        if self.vocab_size < min_vocab_size:
            raise ValueError(
                f"vocab_size is set to {self.vocab_size} but it must be at least {min_vocab_size} to accommodate "
                f"{self.num_codebooks} x {self.codebook_size} codes and {len(self.special_tokens)} special token(s).\n"
                f"Consider setting vocab_size to {min_vocab_size} + K, where K is the number of tokens you want to "
                "reserve for codebook ngrams (learned merges). K should be a sufficiently large number (e.g. >= "
                "10,000) to allow for wide coverage of the most common codebook ngrams in your training data.")
        self._model = None
        self.last_stats: Dict[str, float] = {}
        # the last training's learned tokens (alphabet-index tuples) and merges (left id, right id), ids counted
        # from the special tokens: oracle/bpe_ref.train_bpe's convention
        self.last_tokens: List[Tuple[int, ...]] = []
        self.last_merges: List[Tuple[int, int]] = []

    # ---- corpus ----------------------------------------------------------------------------------
    def iterate_codepoints(self, codes_list: Iterable[np.ndarray]) -> Iterable[np.ndarray]:
        """``_iterate_and_convert`` (bpe_trainer.py:73-105): per utterance, shape handling, first
        num_codebooks rows, chunks of int(chunk_size_secs * codec_framerate) frames -> code points."""
        for codes in codes_list:
            if len(codes.shape) == 4:
                codes = codes[0, 0]
            elif len(codes.shape) == 3:
                codes = codes[0]
            codes = codes[:self.num_codebooks]
            chunk_size = int(self.chunk_size_secs * self.codec_framerate) if self.chunk_size_secs else codes.shape[1]
            for i in range(0, codes.shape[1], chunk_size):
                yield codes_to_codepoints(codes[:, i:i + chunk_size], self.codebook_size,
                                          copy_before_conversion=False, unicode_offset=self.unicode_offset)

    def words(self, codes_list: Iterable[np.ndarray]) -> Tuple[List[np.ndarray], np.ndarray]:
        """Distinct training words (alphabet indices) and their counts."""
        if self._model is None:
            self._model = CharModel(self.unicode_offset, self.num_codebooks * self.codebook_size)
        counts: Dict[bytes, int] = {}
        arrays: Dict[bytes, np.ndarray] = {}
        for cps in self.iterate_codepoints(codes_list):
            for w in self._model.words(cps):
                k = w.astype(np.int32).tobytes()
                if k in counts:
                    counts[k] += 1
                else:
                    counts[k] = 1
                    arrays[k] = w.astype(np.int32)
        keys = list(counts)
        return [arrays[k] for k in keys], np.array([counts[k] for k in keys], dtype=np.int64)

    # ---- training --------------------------------------------------------------------------------
    def _max_token_length(self) -> Optional[int]:
        if self.max_token_codebook_ngrams is None:
            return None
        return max(1, self.max_token_codebook_ngrams * self.num_codebooks)

    def train_codes(self, codes_list: Iterable[np.ndarray]):
        """Train on in-memory code arrays; returns the tokenizer (see ``train``)."""
        n_base = self.num_codebooks * self.codebook_size
        max_len = self._max_token_length()
        if max_len == 1:
            tokens, merges = [], []
        else:
            t0 = time.perf_counter()
            words, counts = self.words(codes_list)
            corpus_s = time.perf_counter() - t0
            # tokenizers treats max_token_length as exclusive: codec_bpe passes the limit + 1
            tokens, merges = train_words_gpu(words, counts, n_base, len(self.special_tokens), self.vocab_size,
                                             self.min_frequency, max_len + 1 if max_len is not None else None,
                                             self.device, self.last_stats)
            self.last_stats["corpus_s"] = corpus_s  # host: chunks -> code points -> words (NFKC model)
        self.last_tokens, self.last_merges = tokens, merges
        t0 = time.perf_counter()
        tok = self._assemble(tokens, merges)
        self.last_stats["assemble_s"] = time.perf_counter() - t0  # tokenizers / transformers objects
        return tok

    def train(self, codes_path: str, codes_filter: Optional[Union[str, List[str]]] = None,
              num_files: Optional[int] = None):
        """``Trainer.train`` (bpe_trainer.py:107-166): BPE over the code files under codes_path."""
        if self._max_token_length() == 1:
            return self._assemble([], [])
        codes_files = get_codes_files(codes_path, codes_filter, num_files)
        if not self.chunk_size_secs and codes_files[0].split("_")[-1].startswith("c"):
            warnings.warn(
                "The codes files do not have start timestamps, indicating they represent full-length encoded audio "
                "files rather than chunks. It is recommended to set `--chunk_size_secs` to a small value (e.g. 30) "
                "to avoid the tokenizer training on very long sequences. Training on very long sequences of audio "
                "codes can lead to memory issues and poor BPE merges.")
        return self.train_codes(u for f in codes_files for u in _utterances(f))

    # ---- output ----------------------------------------------------------------------------------
    def vocab_and_merges(self, tokens: Sequence[Tuple[int, ...]], merges: Sequence[Tuple[int, int]]):
        """token strings in id order and merges as string pairs (tokenizers' BPE model content)."""
        base = self.unicode_offset
        n_base = self.num_codebooks * self.codebook_size
        strs = list(self.special_tokens) + [chr(base + i) for i in range(n_base)]
        strs += ["".join(chr(base + i) for i in t) for t in tokens]
        merge_strs = [(strs[a], strs[b]) for a, b in merges]
        return strs, merge_strs

    def _assemble(self, tokens, merges):
        from tokenizers import Tokenizer, decoders, pre_tokenizers
        from tokenizers.models import BPE
        from tokenizers.normalizers import NFKC
        strs, merge_strs = self.vocab_and_merges(tokens, merges)
        vocab = {}
        for i, s in enumerate(strs):
            vocab.setdefault(s, i)
        tok = Tokenizer(BPE(vocab, merge_strs, unk_token=self.unk_token))
        if self.special_tokens:
            tok.add_special_tokens(list(self.special_tokens))
        tok.normalizer = NFKC()
        tok.pre_tokenizer = pre_tokenizers.Metaspace(replacement="▁", prepend_scheme="never")
        tok.decoder = decoders.Metaspace(replacement="▁", prepend_scheme="never")
        try:
            from transformers import PreTrainedTokenizerFast
        except Exception:  # pragma: no cover - transformers absent: the tokenizers object
            return tok
        return PreTrainedTokenizerFast(tokenizer_object=tok, bos_token=self.bos_token, eos_token=self.eos_token,
                                       unk_token=self.unk_token, pad_token=self.pad_token,
                                       clean_up_tokenization_spaces=False,
                                       model_input_names=["input_ids", "attention_mask"])


def train_words_gpu(words: Sequence[np.ndarray], counts: np.ndarray, n_base: int, n_special: int, vocab_size: int,
                    min_frequency: int, max_token_length: Optional[int], device: int = 0,
                    stats: Optional[dict] = None) -> Tuple[List[Tuple[int, ...]], List[Tuple[int, int]]]:
    """The merge loop on the GPU (``mimi_bpe_*``).  words: alphabet indices (0 .. n_base-1).  Returns
    (tokens beyond the alphabet as tuples of alphabet indices, merges as (left id, right id)) with ids counted
    from the special tokens, as ``oracle/bpe_ref.train_bpe``."""
    import time

    from . import _lib
    lib = _lib.load()
    lens = np.array([len(w) for w in words], dtype=np.int64)
    offs = np.zeros(len(words) + 1, dtype=np.int64)
    np.cumsum(lens, out=offs[1:])
    sym = (np.concatenate(words).astype(np.int32) if len(words) else np.zeros(0, np.int32)) + np.int32(n_special)
    cnt = np.ascontiguousarray(counts, dtype=np.int64)
    if vocab_size > (1 << 17) - 1:
        raise ValueError("vocab_size above 131071 is not supported by the GPU trainer")
    h = ctypes.c_void_p()
    t0 = time.perf_counter()
    _lib.check(lib.mimi_bpe_create(device, sym.ctypes.data, sym.size, offs.ctypes.data, cnt.ctypes.data, len(words),
                                   n_special + n_base, vocab_size, max_token_length or 0, ctypes.byref(h)))
    tokens: List[Tuple[int, ...]] = []
    merges: List[Tuple[int, int]] = []
    spell: List[Tuple[int, ...]] = [()] * n_special + [(i,) for i in range(n_base)]
    tok_id: Dict[Tuple[int, ...], int] = {t: i for i, t in enumerate(spell) if i >= n_special}
    a, b, c = ctypes.c_int32(), ctypes.c_int32(), ctypes.c_int64()
    try:
        while len(spell) < vocab_size:
            _lib.check(lib.mimi_bpe_best(h, ctypes.byref(a), ctypes.byref(b), ctypes.byref(c)))
            if c.value < 1 or c.value < min_frequency:
                break
            new = spell[a.value] + spell[b.value]
            nid = tok_id.get(new)
            if nid is None:
                nid = len(spell)
                spell.append(new)
                tok_id[new] = nid
                tokens.append(new)
            merges.append((a.value, b.value))
            if stats is not None and "trace" in stats:
                stats["trace"].append(c.value)
            _lib.check(lib.mimi_bpe_merge(h, a.value, b.value, nid, len(new)))
    finally:
        lib.mimi_bpe_destroy(h)
    if stats is not None:
        stats.update({"seconds": time.perf_counter() - t0, "merges": len(merges), "symbols": int(sym.size),
                      "words": len(words)})
    return tokens, merges
