"""Diagnostic: first merge where the GPU trainer and the CPU oracle diverge on a synthetic corpus."""
import sys
import os
import heapq
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "tokenize-audio_amd"), ROOT, os.path.join(ROOT, "tests", "golden")]
from make_bpe_golden import CBS, NCB, corpus  # noqa: E402
from mimi_hip import bpe  # noqa: E402
from oracle.bpe_ref import train_bpe  # noqa: E402

n, M = int(sys.argv[1]), int(sys.argv[2])
utts = corpus(seed=9, n_utt=n)
vocab = NCB * CBS + 1 + M
tr = bpe.Trainer(NCB, CBS, codec_framerate=12.5, chunk_size_secs=30, vocab_size=vocab, pad_token="<pad>",
                 max_token_codebook_ngrams=2)
words, counts = tr.words([u.copy() for u in utts])
st = {"trace": []}
gt, gm = bpe.train_words_gpu(words, counts, NCB * CBS, 1, vocab, 2, 17, 0, st)
tr_o = []
ot, om = train_bpe([w + 1 for w in words], counts, NCB * CBS, 1, vocab, 2, 17, trace=tr_o)
print("gpu merges", len(gm), "oracle merges", len(om), "equal", gm == om)
for i, (x, y) in enumerate(zip(gm, om)):
    if x != y:
        print("first diff at", i, "gpu", x, "oracle", y, "gpu counts", st["trace"][:i + 1])
        pc = tr_o[i][1] if i < 3 else None
        if pc is not None:
            print("oracle counts at step", i, "best", tr_o[i][0], "gpu's pair", pc.get(tuple(x)), "oracle's pair", pc.get(tuple(y)))
            print("oracle merges", om[:i + 1])
            top = sorted(pc.items(), key=lambda kv: (-kv[1], kv[0]))[:5]
            print("oracle top", top)
        # recount pair counts after i merges with the oracle to see who is right
        _, om_i = train_bpe([w + 1 for w in words], counts, NCB * CBS, 1, NCB * CBS + 1 + i, 2, 17)
        break
