"""Codec-BPE training time: the GPU trainer (mimi_hip.bpe) vs HF tokenizers' BpeTrainer (the reference's
trainer, CPU, all its threads) on the same synthetic code corpus with the recipe's settings
(codec-bpe/train_bpe_recipe.txt:18-28: 8 codebooks x 2048, 30 s chunks, max_token_codebook_ngrams 2).  Checks
that both give the same merges.

    python tools/bpe_bench.py --utts 400 --merges 8000
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "tokenize-audio_amd"), ROOT, os.path.join(ROOT, "tests", "golden")):
    sys.path.insert(0, p)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--utts", type=int, default=400)
    ap.add_argument("--merges", type=int, default=8000)
    ap.add_argument("--no-reference", action="store_true")
    args = ap.parse_args()
    from make_bpe_golden import CBS, CHUNK, NCB, corpus, train_reference

    from mimi_hip import bpe
    from mimi_hip.codes import codes_to_chars
    utts = corpus(seed=9, n_utt=args.utts)
    frames = sum(u.shape[1] for u in utts)
    vocab = NCB * CBS + 1 + args.merges
    tr = bpe.Trainer(NCB, CBS, codec_framerate=12.5, chunk_size_secs=30, vocab_size=vocab, pad_token="<pad>",
                     max_token_codebook_ngrams=2)
    t0 = time.perf_counter()
    words, counts = tr.words([u.copy() for u in utts])
    t1 = time.perf_counter()
    tokens, merges = bpe.train_words_gpu(words, counts, NCB * CBS, 1, vocab, 2, 17, 0, tr.last_stats)
    t2 = time.perf_counter()
    out = {"frames": frames, "audio_hours": frames / 12.5 / 3600, "symbols": int(sum(len(w) for w in words)),
           "merges": len(merges), "gpu_host_prep_s": round(t1 - t0, 3), "gpu_train_s": round(t2 - t1, 3)}
    if not args.no_reference:
        import multiprocessing
        strings = [codes_to_chars(u[:, i:i + CHUNK], CBS) for u in utts for i in range(0, u.shape[1], CHUNK)]
        t3 = time.perf_counter()
        j = train_reference(strings, vocab, 17)
        t4 = time.perf_counter()
        ref = [tuple(m) for m in j["model"]["merges"]]
        n_sp, n_base = 1, NCB * CBS
        spell = lambda x: chr(0xE000 + x - n_sp) if x < n_sp + n_base else "".join(  # noqa: E731
            chr(0xE000 + i) for i in tokens[x - n_sp - n_base])
        out.update({"tokenizers_train_s": round(t4 - t3, 3), "tokenizers_threads": multiprocessing.cpu_count(),
                    "same_merges": ref == [(spell(a), spell(b)) for a, b in merges]})
    print(json.dumps(out))


if __name__ == "__main__":
    main()
