"""Write the bench's synthetic reference as FASTA (uniform ACGT,
seed 42, records proportional to GRCh38 chromosome lengths, 80 columns).

usage: python tools/make_ref_fasta.py <out.fa> <total bp> <records>
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402  (record_lengths)
import sahara_amd as sa  # noqa: E402


def main(out, total, nrec):
    lens = bench.record_lengths(int(total), int(nrec))
    flat, lens = sa.synth_reference(lens, sigma=6, seed=42)
    chars = np.frombuffer(b"$ACGNT", np.uint8)
    off = 0
    with open(out, "wb") as f:
        for r, L in enumerate(lens.tolist()):
            f.write(b">chr%d synthetic\n" % (r + 1))
            seq = chars[flat[off:off + L]]
            full = L // 80
            if full:
                block = np.empty((full, 81), np.uint8)
                block[:, :80] = seq[:full * 80].reshape(full, 80)
                block[:, 80] = ord("\n")
                f.write(block.tobytes())
            if L % 80:
                f.write(seq[full * 80:].tobytes() + b"\n")
            off += L


if __name__ == "__main__":
    main(*sys.argv[1:])
