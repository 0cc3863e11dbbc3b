#!/usr/bin/env python3
"""Generate tests/golden/tensor_ops.npz (container only).

tests/compat/tensor_ops.cc exercises every xylo/tensor.h operation through
the reference's API only.  `make -C oracle ref` compiles it against the
reference's own tensor.h / tensor.cc (oracle/_ref/tensor_ops_ref, the
reference's flags); this script runs that build and stores its results:

    make -C oracle ref && python tests/golden/make_tensor_golden.py

The drop-in build of the same source (build/compat/tensor_ops) is held to
the fixture by tests/test_tensor_compat.py (host paths, CPU) and
tests/test_gpu_tensor.py (device paths).  Entries: float arrays ("f"),
integer arrays ("i": shapes, indices, flags, engine draws) and strings
("s": streamable output), keyed by result name; `__kinds` maps each name to
its kind.
"""
import os
import subprocess
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF_BIN = os.path.join(REPO, "oracle", "_ref", "tensor_ops_ref")


def parse(text):
    """{name: (kind, value)} of tensor_ops' output lines."""
    out = {}
    for line in text.splitlines():
        if not line.strip():
            continue
        name, kind, rest = line.split(" ", 2)
        if kind == "s":
            out[name] = ("s", rest)
            continue
        parts = rest.split()
        n, vals = int(parts[0]), parts[1:]
        assert len(vals) == n, (name, n, len(vals))
        if kind == "f":
            out[name] = ("f", np.array([float(v) for v in vals], np.float32))
        else:
            out[name] = ("i", np.array([int(v) for v in vals], np.int64))
    return out


def main():
    if not os.path.exists(REF_BIN):
        sys.exit("build the reference first: make -C oracle ref")
    text = subprocess.run([REF_BIN], capture_output=True, text=True,
                          check=True, timeout=300).stdout
    res = parse(text)
    arrays = {"__kinds": np.array(["%s:%s" % (k, v[0]) for k, v in res.items()])}
    for k, (kind, v) in res.items():
        arrays[k] = np.array(v) if kind == "s" else v
    path = os.path.join(HERE, "tensor_ops.npz")
    np.savez_compressed(path, **arrays)
    print("wrote %s (%d results)" % (path, len(res)))


if __name__ == "__main__":
    main()
