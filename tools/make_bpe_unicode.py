"""Unicode data of the codec-BPE trainer's normalizer, as HF ``tokenizers`` 0.22.2 applies it (run here once;
the output is committed as ``tokenize-audio_amd/mimi_hip/data/bpe_unicode.json``).

The reference trains its codec BPE through ``tokenizers``' NFKC normalizer and Metaspace pre-tokenizer
(``codec-bpe/bpe_trainer.py:147-156``; codec_bpe's SentencePieceBPETokenizer = tokenizers'
``implementations/sentencepiece_bpe.py`` with ``max_token_length`` passed to ``BpeTrainer``).  The code
characters ``chr(0xE000 + k*2048 + c)`` run into the CJK-compatibility / presentation-form block (codebook 3:
1,539 of its 2,048 characters change under NFKC, 21 of them into text containing a SPACE, which the Metaspace
pre-tokenizer splits on) and into scripts with combining marks (codebooks 3-7: canonical reordering of adjacent
marks).  ``tokenizers`` carries Unicode tables older than Python 3.10's ``unicodedata`` (13.0): 32 marks of the
code range have a combining class in Python and none in ``tokenizers``.  This script records, for every code
point Python decomposes or gives a non-zero combining class, what ``tokenizers`` does with it:

* ``nfkc``: ``tokenizers`` NFKC of the character alone (only where it differs from the character);
* ``ccc``: the combining class ``tokenizers`` orders it by (Python's class, or 0 where a probe shows that
  ``tokenizers`` does not reorder it).
"""
import json
import os
import sys
import unicodedata

from tokenizers import normalizers

OUT = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tokenize-audio_amd", "mimi_hip",
                   "data", "bpe_unicode.json")


def main():
    n = normalizers.NFKC()
    nfkc, ccc = {}, {}
    acute, sheva = "́", "ְ"  # ccc 230 / 10 in every Unicode version
    for cp in range(0x110000):
        if 0xD800 <= cp < 0xE000:
            continue
        c = chr(cp)
        pc = unicodedata.combining(c)
        if unicodedata.decomposition(c) or pc:
            out = n.normalize_str(c)
            if out != c:
                nfkc[cp] = [ord(x) for x in out]
        if pc:
            # does tokenizers reorder it?  a mark below 230 moves before a preceding acute; one at 230+ stays
            # after a following sheva only if it is a starter to tokenizers
            if pc < 230:
                known = n.normalize_str(acute + c) == c + acute
            else:
                known = n.normalize_str(c + sheva)[0] == sheva
            ccc[cp] = pc if known else 0
    data = {"tokenizers": __import__("tokenizers").__version__, "python_unicodedata": unicodedata.unidata_version,
            "nfkc": {str(k): v for k, v in sorted(nfkc.items())},
            "ccc": {str(k): v for k, v in sorted(ccc.items())}}
    with open(OUT, "w") as f:
        json.dump(data, f, separators=(",", ":"))
    print(f"wrote {OUT}: {len(nfkc)} NFKC entries, {len(ccc)} combining classes "
          f"({sum(1 for v in ccc.values() if v == 0)} unknown to tokenizers)", file=sys.stderr)


if __name__ == "__main__":
    main()
