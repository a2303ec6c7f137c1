"""Static check of the gfx950 device code: every s_barrier must be reached with no LDS write of the wave still in
flight (an s_waitcnt lgkmcnt(0) in between).  hipcc (ROCm 7.2) can drop that wait on a loop's back edge into a
barrier at the loop header -- then a wave on another SIMD may read LDS the writer has not yet updated
(attention_band_h16_kernel's chunk maxima did exactly that, ops.hip).  Scans the straight-line text plus branches
into labels whose first instruction is s_barrier.

    python tools/lds_barrier_scan.py                 # compiles every csrc/*.hip to device asm, scans
    python tools/lds_barrier_scan.py file.s [...]    # scans given asm
"""
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "tokenize-audio_amd", "csrc")
LDS_WRITE = re.compile(r"ds_(write|add|sub|min|max|or|and|xor|inc|dec|cmpst|swap|cmpswap)")


def scan(text):
    lines = text.split("\n")
    barrier_labels = set()
    for i, l in enumerate(lines):
        m = re.match(r"^(\.LBB\w+):", l)
        if m:
            j = i + 1
            while j < len(lines) and (not lines[j].strip() or lines[j].strip().startswith(";")):
                j += 1
            if j < len(lines) and lines[j].strip().startswith("s_barrier"):
                barrier_labels.add(m.group(1))
    bad, fn, pending = [], None, False
    for i, l in enumerate(lines):
        m = re.match(r"^(_Z\w+):", l)
        if m:
            fn, pending = m.group(1), False
            continue
        t = l.strip()
        if LDS_WRITE.match(t):
            pending = True
        elif t.startswith("s_waitcnt") and "lgkmcnt(0)" in t:
            pending = False
        elif t.startswith("s_barrier") and pending:
            bad.append((fn, i + 1, "falls into s_barrier"))
        elif (t.startswith("s_branch") or t.startswith("s_cbranch")) and pending and t.split()[-1] in barrier_labels:
            bad.append((fn, i + 1, "branches to " + t.split()[-1]))
    return bad


def compile_all(out_dir):
    outs = []
    for f in sorted(os.listdir(CSRC)):
        if not f.endswith(".hip"):
            continue
        o = os.path.join(out_dir, f + ".s")
        subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-ffp-contract=off", "--offload-arch=gfx950",
                        "-I", CSRC, "--cuda-device-only", "-S", os.path.join(CSRC, f), "-o", o],
                       check=True, capture_output=True)
        outs.append(o)
    return outs


def main(argv):
    if argv:
        files = argv
    else:
        tmp = tempfile.mkdtemp()
        files = compile_all(tmp)
    bad = []
    for f in files:
        bad += [(os.path.basename(f),) + b for b in scan(open(f).read())]
    for b in bad:
        print(*b)
    print(f"{len(files)} files, {len(bad)} barriers with LDS writes in flight")
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
