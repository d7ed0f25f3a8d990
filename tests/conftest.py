"""Test configuration.

* ``gpu`` marker: needs a real MI355X (run with ``-m gpu`` on the GPU box).
* Paths: the repo root (``oracle`` package) and ``grape-vector-db_amd``
  (``gvdb`` package) are importable.
* The CPU oracle (test infrastructure) is built on demand; libgvdb.so is built
  by ``__graft_entry__.build()`` (the ABI tests build it when missing).
"""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "grape-vector-db_amd")
for p in (ROOT, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X GPU (HIP device)")


@pytest.fixture(scope="session")
def oracle_mod():
    import oracle

    oracle.lib()
    return oracle


@pytest.fixture(scope="session")
def gvdb_lib_path():
    so = os.path.join(PKG, "libgvdb.so")
    if not os.path.exists(so):
        subprocess.run(["make", "-s", "-C", PKG, "-j8"], check=True)
    return so


@pytest.fixture(scope="session")
def gvdb_mod(gvdb_lib_path):
    import gvdb

    gvdb.lib()
    return gvdb
