"""bjxa_hip_parse_headers_async (include/bjxa_hip.h) against the oracle's
restatement of bjxa_parse_header (src/libbjxa.c:395-453): every record field
and status, bit-exact, on seeded random valid and broken headers, the
golden files' headers, unaligned strides and ragged counts."""
import numpy as np
import pytest
import torch

import bjxa_amd
import oracle

pytestmark = pytest.mark.gpu

FIELDS = ("data_len", "samples", "blocks", "data_len_pcm", "rate", "bits", "channels")


def run(hdrs, stride):
    n = hdrs.shape[0]
    buf = np.zeros(max(n * stride, 1), np.uint8)
    for i in range(n):
        buf[i * stride:i * stride + 32] = hdrs[i]
    d_src = torch.from_numpy(buf).cuda()
    dt = bjxa_amd.header_record()
    d_out = torch.full((max(n, 1) * dt.itemsize,), 0xAB, dtype=torch.uint8, device="cuda")
    bjxa_amd.parse_headers_device(d_src.data_ptr(), stride, n, d_out.data_ptr(),
                                  torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    return np.frombuffer(d_out.cpu().numpy().tobytes(), dt)[:n]


def check(hdrs, rec):
    for h, r in zip(hdrs, rec):
        want = oracle.validate_xa_header(h)
        if want is None:
            assert r["status"] == 71, h.tobytes()            # EPROTO
            assert all(int(r[f]) == 0 for f in FIELDS) and not r["state"].any()
        else:
            assert r["status"] == 0, h.tobytes()
            for f in FIELDS:
                assert int(r[f]) == want[f], (f, h.tobytes())
            assert tuple(int(v) for v in r["state"]) == want["state"]


@pytest.mark.parametrize("stride,n", [(32, 100_000), (33, 4097), (47, 1), (4096, 300)])
def test_random_headers(built, stride, n):
    rng = np.random.default_rng(stride * 7 + n)
    hdrs = oracle.random_xa_headers(rng, min(n, 20_000))
    if n > hdrs.shape[0]:
        hdrs = np.concatenate([hdrs] * (-(-n // hdrs.shape[0])))[:n]
    rec = run(hdrs, stride)
    check(hdrs[:20_000], rec[:20_000])
    if n > 20_000:      # the repeats decode the same as their first copy
        assert np.array_equal(rec[20_000:].view(np.uint8),
                              rec[:n - 20_000].view(np.uint8))


def test_golden_headers(built, golden):
    names = ["square-mono-4.xa", "square-mono-6.xa", "square-mono-8.xa",
             "square-stereo-4.xa", "square-stereo-6.xa", "square-stereo-8.xa"]
    hdrs = np.stack([np.frombuffer(golden(nm)[:32], np.uint8) for nm in names])
    rec = run(hdrs, 32)
    check(hdrs, rec)
    assert (rec["status"] == 0).all()


def test_odd_stereo_is_eproto(built):
    bs = 33
    h = np.frombuffer(bjxa_amd.xa_header(3 * bs, 48, 44100, 8, 2), np.uint8)[None]
    assert run(h, 32)[0]["status"] == 71


def test_empty_and_bad_args(built):
    assert bjxa_amd.lib().bjxa_hip_parse_headers_async(None, 32, 0, None, None) == 0
    assert bjxa_amd.lib().bjxa_hip_parse_headers_async(None, 32, 1, None, None) == -1
    assert bjxa_amd.lib().bjxa_hip_parse_headers_async(1, 31, 1, 1, None) == -1
