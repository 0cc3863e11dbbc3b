#!/usr/bin/env python3
"""Golden outputs of the drop-in layer's test programs (tests/compat/*.cc) as
the REAL reference runs them: each program is compiled against the reference
headers under /root/reference with the reference flags and linked with the
reference's own tensor.cc / logging.cc objects (oracle/_ref, `make -C oracle
ref`); its stdout lines are stored in tests/golden/<program>.npz.  Container
only (the reference tree does not exist on the GPU box).

    python tests/golden/make_compat_golden.py [program ...]
"""
import os
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"
CXX = "/opt/rocm/lib/llvm/bin/clang++"
FLAGS = ["-O3", "-std=c++20", "-mavx", "-ffast-math", "-I" + REF]
OBJS = [os.path.join(REPO, "oracle", "_ref", o) for o in ("tensor.o", "logging.o")]
PROGRAMS = ["bound_env_by_hand"]


def main(names):
    for o in OBJS:
        if not os.path.exists(o):
            sys.exit("build the reference objects first: make -C oracle ref")
    for name in names or PROGRAMS:
        src = os.path.join(REPO, "tests", "compat", name + ".cc")
        with tempfile.TemporaryDirectory() as td:
            exe = os.path.join(td, name)
            subprocess.run([CXX] + FLAGS + [src] + OBJS + ["-lpthread", "-o", exe],
                           check=True)
            out = subprocess.run([exe], capture_output=True, text=True,
                                 check=True, timeout=600).stdout
        path = os.path.join(HERE, name + ".npz")
        np.savez_compressed(path, lines=np.array(out.splitlines()))
        print("%-20s %d lines" % (name, len(out.splitlines())))


if __name__ == "__main__":
    main(sys.argv[1:])
