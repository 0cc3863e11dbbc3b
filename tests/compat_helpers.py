"""Helpers for the drop-in C++ layer tests (include/xylo_compat)."""
import os
import re
import subprocess

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
COMPAT = os.path.join(REPO, "build", "compat")
CXX = "/opt/rocm/lib/llvm/bin/clang++"
FLAGS = ["-std=c++20", "-O2", "-Wall", "-Wno-unused-variable",
         "-I" + os.path.join(REPO, "include", "xylo_compat"),
         "-I" + os.path.join(REPO, "include")]
LIBDIR = os.path.join(REPO, "dependence_free_rl_amd")
LINK = ["-L" + LIBDIR, "-lxylo_hip", "-Wl,-rpath," + LIBDIR]
ROUND = re.compile(r"round (\d+) ([-+0-9.eE]+)")


def compile_cc(src, out, extra=()):
    subprocess.run([CXX] + FLAGS + list(extra) + [src] + LINK + ["-o", out],
                   check=True, capture_output=True, text=True)
    return out


def app(name):
    """A driver built by `make compat` (reference apps need /root/reference at
    build time; the built binaries travel with the tree)."""
    return os.path.join(COMPAT, name)


def read_rounds(cmd, n, env, cwd=None, timeout=300):
    """Run a driver until it has logged n 'round k X' lines (n=None: until it
    exits by itself); returns [(k, X)] and the captured stderr text."""
    p = subprocess.Popen(cmd, stderr=subprocess.PIPE, stdout=subprocess.DEVNULL,
                         text=True, env=env, cwd=cwd)
    got, text = [], []
    try:
        import threading
        timer = threading.Timer(timeout, p.kill)
        timer.start()
        for line in p.stderr:
            text.append(line)
            m = ROUND.search(line)
            if m:
                got.append((int(m.group(1)), float(m.group(2))))
                if n is not None and len(got) >= n:
                    break
        timer.cancel()
    finally:
        p.kill()
        p.wait()
    return got, "".join(text)


def fmt6(x):
    """std::ostream's default float formatting (precision 6, %g)."""
    return float("%g" % x)


# ------------------------------------------------ xylo/tensor.h fixtures --
def parse_tensor_ops(text):
    """{name: value} of tests/compat/tensor_ops.cc's output: float32 / int64
    arrays, or strings."""
    import numpy as np
    out = {}
    for line in text.splitlines():
        if not line.strip():
            continue
        name, kind, rest = line.split(" ", 2)
        if kind == "s":
            out[name] = rest
            continue
        parts = rest.split()
        n, vals = int(parts[0]), parts[1:]
        assert len(vals) == n, (name, n, len(vals))
        out[name] = (np.array([float(v) for v in vals], np.float32) if kind == "f"
                     else np.array([int(v) for v in vals], np.int64))
    return out


def tensor_ops_mismatches(text, tol=1e-4):
    """tensor_ops output against tests/golden/tensor_ops.npz (the reference's
    own build of the same source): integers (shapes, indices, flags, engine
    draws) and strings bit-exact, floats within tol * max(1, |y|).  Returns
    [(name, detail)] of the mismatches and the worst float error."""
    import numpy as np
    g = np.load(os.path.join(REPO, "tests", "golden", "tensor_ops.npz"))
    kinds = dict(k.split(":") for k in g["__kinds"])
    got = parse_tensor_ops(text)
    bad = [(k, "missing") for k in kinds if k not in got]
    bad += [(k, "unexpected") for k in got if k not in kinds]
    worst = 0.0
    for k, kind in kinds.items():
        if k not in got:
            continue
        y, x = g[k], got[k]
        if kind == "s":
            if str(y) != x:
                bad.append((k, "%r != %r" % (x, str(y))))
        elif kind == "i":
            if not np.array_equal(x, y):
                bad.append((k, "ints differ"))
        else:
            if x.shape != y.shape:
                bad.append((k, "shape %s != %s" % (x.shape, y.shape)))
                continue
            err = np.abs(x.astype(np.float64) - y) / np.maximum(1.0, np.abs(y))
            e = float(err.max()) if err.size else 0.0
            worst = max(worst, e)
            if not e <= tol:
                bad.append((k, "err %.3g" % e))
    return bad, worst
