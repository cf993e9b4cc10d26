"""The library's build id: the first 16 hex digits of the SHA-256 over the
product sources (sahara_amd/csrc/*.hip, *.cpp, *.h and include/sahara_hip.h,
in byte order of their paths, each as path NUL content NUL). The Makefile
compiles it into libsahara_hip.so (sahara_build_id()); profile summaries
record it, and bench.py marks a committed profile of another build stale.

usage: python tools/build_id.py [repo root]    -> prints the id
"""
import glob
import hashlib
import os
import sys


def build_id(root):
    files = sorted(glob.glob(os.path.join(root, "sahara_amd", "csrc", "*.hip"))
                   + glob.glob(os.path.join(root, "sahara_amd", "csrc", "*.cpp"))
                   + glob.glob(os.path.join(root, "sahara_amd", "csrc", "*.h"))
                   + [os.path.join(root, "include", "sahara_hip.h")],
                   key=lambda p: os.path.relpath(p, root).encode())
    h = hashlib.sha256()
    for f in files:
        h.update(os.path.relpath(f, root).encode() + b"\0")
        h.update(open(f, "rb").read() + b"\0")
    return h.hexdigest()[:16]


if __name__ == "__main__":
    print(build_id(sys.argv[1] if len(sys.argv) > 1 else os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
