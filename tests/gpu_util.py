"""Device-side helpers shared by the GPU tests (torch provides HBM buffers
and the stream; all compute goes through libbjxa.so.0's C-ABI)."""
import numpy as np

import bjxa_amd


def require_gpu():
    import torch
    assert torch.cuda.is_available(), "GPU test run without a visible GPU"
    return torch


def dev_decode(xa, eblocks, bits, ch, frames=None, state=(0, 0, 0, 0), chunk=0, warmup=-1,
               want_status=False, variant=0):
    """Decode host XA bytes through bjxa_hip_decode_async; returns int16 PCM."""
    torch = require_gpu()
    if frames is None:
        frames = eblocks * 32
    src = torch.from_numpy(np.ascontiguousarray(xa, dtype=np.uint8)).cuda()
    dst = torch.full((eblocks * 64 * ch,), 0x5A, dtype=torch.uint8, device="cuda")
    ws_len = bjxa_amd.decode_workspace_size(eblocks, ch, chunk, warmup, variant)
    ws = torch.zeros(ws_len, dtype=torch.uint8, device="cuda")
    status = torch.zeros(bjxa_amd.STATUS_WORDS, dtype=torch.int32, device="cuda")
    stream = torch.cuda.current_stream().cuda_stream
    bjxa_amd.workspace_init(ws.data_ptr(), ws_len, stream)
    bjxa_amd.decode_device(src.data_ptr(), dst.data_ptr(), eblocks, frames, bits, ch,
                           ws.data_ptr(), ws_len, status.data_ptr(), state, chunk, warmup,
                           stream, variant=variant)
    torch.cuda.synchronize()
    out = dst.cpu().numpy()
    pcm = out.view(np.int16)[:frames * ch].copy()
    st = status.cpu().numpy().view(np.uint32).copy()
    # bytes past the emitted frames must be untouched
    assert (out[frames * ch * 2:] == 0x5A).all()
    if want_status:
        return pcm, st
    return pcm


def status_state(st):
    def split(w):
        w = int(w)
        return [np.int16(np.uint16(w & 0xFFFF)), np.int16(np.uint16(w >> 16))]
    return tuple(int(v) for v in split(st[1]) + split(st[2]))


def dev_encode(pcm, frames, bits, ch):
    torch = require_gpu()
    src = torch.from_numpy(np.ascontiguousarray(pcm, dtype=np.int16)).cuda()
    eblocks = (frames + 31) // 32
    n = eblocks * ch * (bits * 4 + 1)
    dst = torch.full((n + 64,), 0xA5, dtype=torch.uint8, device="cuda")
    bjxa_amd.encode_device(src.data_ptr(), frames, bits, ch, dst.data_ptr(),
                           torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    out = dst.cpu().numpy()
    assert (out[n:] == 0xA5).all()
    return out[:n].copy()
