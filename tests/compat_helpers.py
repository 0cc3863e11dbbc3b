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
