"""One XA stream split over several GPUs.

Each rank owns a contiguous range of effective blocks [lo, hi) and decodes
it on its own GPU, speculatively: it warms up over the `warmup` eblocks
before its range from state (0, 0) -- the same speculation the kernels use
between chunks -- so it needs those eblocks in its input too.  One
all-gather then exchanges every rank's (entry state used, exit state
reached); the true entry state of rank r is rank r-1's true exit state
(rank 0: the stream's initial state).  A rank whose entry state was wrong
re-decodes its range from the true one, and the exchange repeats until the
chain is consistent: each round settles at least the first wrong rank, and
in practice one round settles all (a wrong entry state meets the true
trajectory within a few blocks, so the re-decode's exit state is right).

The protocol (`resolve`) is independent of how a range is decoded: the
product passes the GPU decode (`device_range_decoder`); the CPU test passes
the oracle.  States are packed like the kernels' (p0 | p1 << 16 per
channel, L then R).
"""
import numpy as np


def split_ranges(eblocks, world):
    """Contiguous, balanced [lo, hi) per rank."""
    return [(r * eblocks // world, (r + 1) * eblocks // world) for r in range(world)]


def _pack(state):
    """(L p0, L p1, R p0, R p1) int16 -> two packed words."""
    s = [int(np.uint16(np.int16(v))) for v in state]
    return (s[0] | (s[1] << 16), s[2] | (s[3] << 16))


def _unpack(words):
    out = []
    for w in words:
        out += [int(np.int16(np.uint16(w & 0xFFFF))), int(np.int16(np.uint16(w >> 16)))]
    return tuple(out)


NO_ERROR = 1 << 62


def resolve(local_decode, lo, hi, init_state, warmup, group=None):
    """Run the split-decode protocol for this rank's range [lo, hi).

    local_decode(first, state) decodes eblocks [first, hi) of the stream
    starting from `state` and returns (state at lo, exit state at hi) or
    (state at lo, exit state, bad), where bad is the stream-global index
    (eblock * channels + channel) of the first channel block in [lo, hi)
    whose gain nibble is >= 5, and the exit state is then the one the
    reference carries out of a failing call: the state after the last
    good eblock, with the left channel of the bad eblock applied when the
    right block is the bad one (src/libbjxa.c:633-643).  It is called with
    first = max(lo - warmup, 0) and state (0,0,0,0) for the speculative
    pass (the stream's init_state when first == 0), and with first = lo and
    the true entry state for a re-decode.  Its PCM output for [lo, hi)
    must be left in place by the last call.

    Returns (exit state, bad): the stream's exit state and None, or -- the
    reference's first-bad-block semantics -- the carried state at the first
    bad channel block of the whole stream and its index (every rank gets
    the same value).  Ranks after the failing one are never re-decoded;
    their PCM lies past the error.
    """
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)

    def call(first, state):
        res = tuple(local_decode(first, state))
        g, e = res[0], res[1]
        bad = res[2] if len(res) > 2 and res[2] is not None else NO_ERROR
        return g, e, bad

    first = max(lo - warmup, 0)
    g, e, bad = call(first, init_state if first == 0 else (0, 0, 0, 0))
    if rank == 0:
        g = init_state          # the true entry state, by definition

    def pack(g, e, bad):
        return torch.tensor(list(_pack(g)) + list(_pack(e)) + [bad], dtype=torch.int64)
    mine = pack(g, e, bad)
    true_init = torch.tensor(list(_pack(init_state)), dtype=torch.int64)
    while True:
        parts = [torch.zeros(5, dtype=torch.int64) for _ in range(world)]
        dist.all_gather(parts, mine, group=group)
        # walk the chain: the first rank whose entry state differs from its
        # predecessor's exit must re-decode; later ranks wait for it.  The
        # walk ends at the first rank that holds a bad block.
        t = true_init
        redo = None
        for r in range(world):
            if not torch.equal(parts[r][:2], t):
                redo = r
                break
            if int(parts[r][4]) != NO_ERROR:
                return _unpack([int(v) for v in parts[r][2:4]]), int(parts[r][4])
            t = parts[r][2:4]
        if redo is None:
            return _unpack([int(v) for v in parts[world - 1][2:4]]), None
        if rank == redo:
            g = _unpack([int(v) for v in t])
            _, e, bad = call(lo, g)
            mine = pack(g, e, bad)


def device_range_decoder(d_src_range, d_dst_range, lo, hi, frames, bits, channels,
                         warmup, stream=0):
    """local_decode for `resolve` on the GPU (bjxa_hip_decode_async).

    d_src_range / d_dst_range hold eblocks [max(lo - warmup, 0), hi) of
    the stream (XA in, PCM out), so the rank's own PCM starts
    min(lo, warmup) eblocks into d_dst_range; frames is the stream's total
    frame count (the last rank's range may end in a cut block)."""
    import torch
    import bjxa_amd
    ch = channels
    w0 = max(lo - warmup, 0)
    ebsz = (bits * 4 + 1) * ch

    def frame_state(dst, eblock, first, chans):
        """(p0, p1) of each channel in `chans` after eblock `eblock` (its
        frames 30, 31), from the PCM decoded from eblock `first` on"""
        off = (eblock - first) * 64 * ch + 30 * 2 * ch
        f = device_bytes(dst + off, 4 * ch).view(np.int16).reshape(2, ch)
        return {c: (int(f[1][c]), int(f[0][c])) for c in chans}

    keep = []      # the latest full-block scratch PCM of a cut last block

    def run(first, state):
        """Decode [first, hi) from `state`.  Always whole blocks (as
        bjxa__gpu_decode does): when the stream's last block is cut, the
        range decodes into a full-block scratch buffer and only the
        stream's frames are copied to the caller's PCM, so frames 30/31 of
        every block -- the carried state of a bad right block in the last
        eblock included -- are real (round-2 ADVICE)."""
        n = hi - first
        fr = min(frames, hi * 32) - first * 32
        src = d_src_range + (first - w0) * ebsz
        dst = d_dst_range + (first - w0) * 64 * ch
        out = dst
        if fr < n * 32:
            full = torch.empty(n * 64 * ch, dtype=torch.uint8, device="cuda")
            keep[:] = [full]      # decode() reads frame states from the latest only
            out = full.data_ptr()
        ws_len = bjxa_amd.decode_workspace_size(n, ch)
        ws = torch.zeros(ws_len, dtype=torch.uint8, device="cuda")
        st = torch.zeros(bjxa_amd.STATUS_WORDS, dtype=torch.int32, device="cuda")
        bjxa_amd.workspace_init(ws.data_ptr(), ws_len, stream)
        bjxa_amd.decode_device(src, out, n, n * 32, bits, ch, ws.data_ptr(), ws_len,
                               st.data_ptr(), state, stream=stream)
        torch.cuda.synchronize()
        if out != dst:
            device_copy(dst, out, fr * 2 * ch)
        return out, st.cpu().numpy().view(np.uint32).copy()

    def decode(first, state):
        dst, words = run(first, state)
        if first == lo:
            at_lo = state
        else:
            # state at lo: frames 30, 31 of eblock lo - 1 are (p1, p0)
            s = frame_state(dst, lo - 1, first, range(ch))
            at_lo = tuple(v for c in range(2) for v in (s[c] if c < ch else (0, 0)))
        err = int(words[0])
        if err != bjxa_amd.NO_ERROR and first + err // ch < lo:
            # the first bad block lies in the warm-up, which is the previous
            # rank's to report: look for one in [lo, hi) from lo
            dst, words = run(lo, at_lo)
            first, err = lo, int(words[0])
        if err == bjxa_amd.NO_ERROR:
            return at_lo, _unpack([int(words[1]), int(words[2])]), None
        # the reference stops before the failing eblock j; a bad right
        # block leaves the left channel advanced through eblock j
        j, bad_c = first + err // ch, err % ch
        carried = {c: (v[2 * c], v[2 * c + 1]) for c, v in ((c, at_lo) for c in range(ch))}
        if j > first:
            carried.update(frame_state(dst, j - 1, first, range(ch)))
        if ch == 2 and bad_c == 1:
            carried.update(frame_state(dst, j, first, [0]))
        out = tuple(v for c in range(2) for v in (carried[c] if c < ch else (0, 0)))
        return at_lo, out, j * ch + bad_c

    return decode


_HIP = []


def _hip():
    """libamdhip64 through ctypes, loaded once (the runtime torch already
    brought in)."""
    if not _HIP:
        import ctypes
        hip = ctypes.CDLL("libamdhip64.so.7")
        hip.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t,
                                  ctypes.c_int]
        _HIP.append(hip)
    return _HIP[0]


def device_copy(d_to, d_from, nbytes):
    """hipMemcpy device to device (synchronous)."""
    if nbytes and _hip().hipMemcpy(d_to, d_from, nbytes, 3) != 0:
        raise RuntimeError("hipMemcpy failed")


def device_bytes(d_ptr, nbytes):
    """Copy nbytes from device pointer d_ptr into a host numpy array."""
    out = np.empty(nbytes, dtype=np.uint8)
    if _hip().hipMemcpy(out.ctypes.data, d_ptr, nbytes, 2) != 0:
        raise RuntimeError("hipMemcpy failed")
    return out
