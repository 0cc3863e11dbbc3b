"""CPU check of the wave-specialised train kernel's LDS image layout
(dependence_free_rl_amd/csrc/spec8_layout.h): tests/spec8_layout_check.cc
compiled with the host compiler checks that the layout is a bijection, that
every lane base + loop immediate the kernel uses addresses the element its
MFMA operand map or C layout asks for, and the bank-conflict counts per
access pattern (MI355X_MICROARCH.md §LDS rules): 8-byte stores 2-way (the
minimum for 16 lanes of one half), 16-byte chunk stores 2-way (8 x 8 lanes,
banks mod 32), row and transposed reads conflict-free; for the images of
policy_spec8_kernels.hip and policy_spec4_kernels.hip."""
import os
import subprocess

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_spec8_layout(tmp_path):
    exe = str(tmp_path / "spec8_layout_check")
    subprocess.run(["g++", "-O1", "-std=c++17",
                    "-I" + os.path.join(REPO, "dependence_free_rl_amd", "csrc"),
                    os.path.join(REPO, "tests", "spec8_layout_check.cc"), "-o", exe],
                   check=True)
    out = subprocess.run([exe], capture_output=True, text=True)
    print(out.stdout)
    assert out.returncode == 0, out.stdout + out.stderr
    assert "stores: 2-way" in out.stdout
    assert "row reads: 1-way" in out.stdout
    assert "transposed reads: 1-way" in out.stdout
    assert "chunk stores: 2-way" in out.stdout
    assert "column order: ok" in out.stdout
