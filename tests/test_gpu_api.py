"""The C API contract test (tests/c/test_api.c) with the GPU present."""
import os
import subprocess

import pytest

from conftest import GOLDEN
from test_abi import build_api_test

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("offload", ["0", None])
def test_c_api_contract_gpu(built, manifest, tmp_path, offload):
    """The same contract with the GPU visible: every call on the kernels
    (offload threshold 0), and with the default routing."""
    import hashlib
    exe = build_api_test(built, tmp_path)
    env = dict(os.environ)
    if offload is not None:
        env.update(BJXA_OFFLOAD_DECODE=offload, BJXA_OFFLOAD_ENCODE=offload)
    wav = tmp_path / "out.wav"
    r = subprocess.run([exe, GOLDEN, str(wav)], stdin=subprocess.DEVNULL, capture_output=True,
                       text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr
    assert "test_api: ok" in r.stdout
    sha = hashlib.sha1(wav.read_bytes()).hexdigest()
    assert sha == manifest["fixtures"]["square-mono-4.xa"]["wav_sha1"]
