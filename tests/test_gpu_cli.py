"""The reference's CLIs over the C-ABI (bo-lz4-ada_amd/unlz4ada,
bo-lz4-ada_amd/xxhash32ada), run the way test_run.sh runs the reference's
tool_unlz4ada: every .lz4 vector through stdin, sha256 of stdout against
the vector's expected output, exit status 0 (test_run.sh:13-40); error
vectors end with the reference's exception line and a non-zero status."""
import hashlib
import os
import subprocess

import pytest

import _oracle as O
from conftest import PKG, VECTORS, error_vectors, good_vectors, read_vector

pytestmark = pytest.mark.gpu

UNLZ4 = os.path.join(PKG, "unlz4ada")
XXH = os.path.join(PKG, "xxhash32ada")


def run(exe, data, *args):
    return subprocess.run([exe, *args], input=data, capture_output=True, timeout=120)


@pytest.mark.parametrize("name", good_vectors())
def test_unlz4ada_good_vectors(name, digests):
    # config[0] of BASELINE.json is z100 through this path
    p = run(UNLZ4, read_vector(name, "lz4"))
    assert p.returncode == 0, p.stderr.decode()
    assert len(p.stdout) == digests[name]["len"]
    assert hashlib.sha256(p.stdout).hexdigest() == digests[name]["sha256"]


def test_unlz4ada_file_argument(digests):
    p = subprocess.run([UNLZ4, os.path.join(VECTORS, "t1111k.lz4")], capture_output=True, timeout=120)
    assert p.returncode == 0
    assert hashlib.sha256(p.stdout).hexdigest() == digests["t1111k"]["sha256"]


@pytest.mark.parametrize("name", error_vectors())
def test_unlz4ada_error_vectors(name):
    data = read_vector(name, "err")
    st, ref, msg = O.unlz4ada(data)
    p = run(UNLZ4, data)
    assert p.returncode == 1
    assert p.stderr.decode().strip() == O.exception_information(st, msg)
    assert p.stdout == ref  # what the reference wrote before raising, block by block


def test_xxhash32ada():
    data = read_vector("t1111k", "lz4")
    p = run(XXH, data)
    assert p.returncode == 0
    assert p.stdout.decode() == "xxhash32(0, stdin) = 0x%08x\n" % O.xxh32(data)
    p = run(XXH, b"")
    assert p.stdout.decode() == "xxhash32(0, stdin) = 0x02cc5d05\n"


UNLZ4S = os.path.join(PKG, "unlz4ada_simple")


@pytest.mark.parametrize("name", good_vectors())
def test_unlz4ada_simple_good_vectors(name, digests):
    """tool_unlz4ada_simple: Init(For_All) + Update over 4 KiB reads (the
    streaming facade on the GPU), every vector incl. concatenated frames."""
    p = run(UNLZ4S, read_vector(name, "lz4"))
    assert p.returncode == 0, p.stderr.decode()
    assert hashlib.sha256(p.stdout).hexdigest() == digests[name]["sha256"]


@pytest.mark.parametrize("name", error_vectors())
def test_unlz4ada_simple_error_vectors(name):
    data = read_vector(name, "err")
    st, ref, eof, msg = O.decode_stream(data, chunk=4096, reservation=O.FOR_ALL)
    p = run(UNLZ4S, data)
    if st == O.OK:
        # For_All accepts what Single_Frame rejects (e.g. trailing bytes as a
        # next frame); then the tool's own end-of-input check decides
        assert p.stdout == ref
        if eof == O.EOF_NO:
            assert p.returncode == 1
            assert p.stderr.decode().strip() == "raised CONSTRAINT_ERROR : Input ended mid-frame."
        else:
            assert p.returncode == 0
    else:
        assert p.returncode == 1
        assert p.stderr.decode().strip() == O.exception_information(st, msg)
        assert ref.startswith(p.stdout)
