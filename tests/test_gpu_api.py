"""The C API contract test (tests/c/test_api.c) with the GPU present."""
import os
import subprocess

import pytest

from conftest import GOLDEN
from test_abi import build_api_test

pytestmark = pytest.mark.gpu


def test_c_api_contract_gpu(built, tmp_path):
    exe = build_api_test(built, tmp_path)
    r = subprocess.run([exe, GOLDEN, "gpu"], stdin=subprocess.DEVNULL, capture_output=True,
                       text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    assert "test_api: ok" in r.stdout
