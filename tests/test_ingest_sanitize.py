"""Sanitizer builds of the multi-threaded Matrix Market reader (csrc/mtx.cpp, host code only):
AddressSanitizer + UndefinedBehaviorSanitizer and ThreadSanitizer executables built with g++
from the library source and tests/native/mtx_sanitize_main.cpp, run over files of every
field/symmetry, multi-chunk sizes, whitespace variants and malformed input at 1, 3 and 8
threads.  Each run must exit cleanly with no sanitizer report and agree with
scipy.io.mmread (the reference's reader, gflownet/utils.py:54-63): dims, entry count and a
fixed-order checksum of the (row, col, value) arrays."""
import os
import shutil
import subprocess

import numpy as np
import pytest
import scipy.io
import scipy.sparse as sp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = [os.path.join(ROOT, "gflownet_spai_amd", "csrc", "mtx.cpp"), os.path.join(ROOT, "tests", "native",
                                                                               "mtx_sanitize_main.cpp")]
FLAGS = {"asan": ["-fsanitize=address,undefined", "-fno-omit-frame-pointer", "-fno-sanitize-recover=all"],
         "tsan": ["-fsanitize=thread"]}
ENV = {"ASAN_OPTIONS": "detect_leaks=1:halt_on_error=1:abort_on_error=0",
       "UBSAN_OPTIONS": "halt_on_error=1:print_stacktrace=1", "TSAN_OPTIONS": "halt_on_error=1"}

pytestmark = pytest.mark.skipif(shutil.which("g++") is None, reason="g++ not available")


@pytest.fixture(scope="module")
def exes(tmp_path_factory):
    d = tmp_path_factory.mktemp("mtx_san")
    out = {}
    for kind, fl in FLAGS.items():
        exe = str(d / f"mtx_{kind}")
        r = subprocess.run(["g++", "-O1", "-g", "-std=c++17", "-pthread", *fl, *SRC, "-o", exe],
                           capture_output=True, text=True)
        if r.returncode != 0:
            pytest.skip(f"{kind} build failed: {r.stderr[-400:]}")
        out[kind] = exe
    return out


def run(exe, path, threads):
    env = dict(os.environ, **ENV)
    r = subprocess.run([exe, path, str(threads)], capture_output=True, text=True, env=env, timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    assert "Sanitizer" not in r.stderr and "runtime error" not in r.stderr, r.stderr[-2000:]
    return r.stdout.split()


def expect(path):
    m = scipy.io.mmread(path).tocoo()
    r, c, v = m.row.astype(np.float64), m.col.astype(np.float64), m.data.astype(np.float64)
    cs = np.cumsum(r * 31.0 + c * 7.0 + v)[-1] if len(r) else 0.0  # sequential, as the harness
    return m.shape, len(r), cs


def files(tmp_path):
    rng = np.random.default_rng(0)
    out = []
    for i, (field, sym) in enumerate([("real", "general"), ("real", "symmetric"), ("integer", "skew-symmetric"),
                                      ("pattern", "general"), ("real", "general")]):
        n = 4000 if i == 4 else 300  # the last one spans many reader chunks
        m = sp.random(n, n, density=0.02 if i == 4 else 0.05, random_state=i, format="coo")
        if sym != "general":
            m = sp.tril(m, k=-1 if sym == "skew-symmetric" else 0).tocoo()
        lines = []
        for a, b, v in zip(m.row, m.col, m.data):
            val = "" if field == "pattern" else (f" {int(v * 100) - 50}" if field == "integer" else f" {v!r}")
            sep = "\t " if (a + b) % 3 == 0 else " "  # whitespace variants
            lines.append(f"{a + 1}{sep}{b + 1}{val}")
        p = tmp_path / f"m{i}.mtx"
        p.write_text(f"%%MatrixMarket matrix coordinate {field} {sym}\n% comment\n%\n{n} {n} {len(lines)}\n"
                     + "\n".join(lines) + "\n")
        out.append(str(p))
    bad = tmp_path / "bad.mtx"
    bad.write_text("%%MatrixMarket matrix coordinate real general\n3 3 2\n1 1 1.0\n2 x 3.0\n")
    out.append(str(bad))
    trunc = tmp_path / "trunc.mtx"
    trunc.write_text("%%MatrixMarket matrix coordinate real general\n5 5 4\n1 1 1.0\n2 2")
    out.append(str(trunc))
    return out


@pytest.mark.parametrize("kind", ["asan", "tsan"])
def test_mtx_reader_under_sanitizers(exes, tmp_path, kind):
    for path in files(tmp_path):
        try:
            ref = expect(path)
        except Exception:  # malformed: the reader must fail cleanly (an error line, no report)
            ref = None
        for threads in (1, 3, 8):
            got = run(exes[kind], path, threads)
            if ref is None or got[0] == "error":
                assert ref is None or got[0] != "error", (path, got)
                continue
            (rows, cols), nnz, cs = ref
            assert (int(got[0]), int(got[1]), int(got[2])) == (rows, cols, nnz), (path, threads)
            assert float(got[3]) == cs, (path, threads)
