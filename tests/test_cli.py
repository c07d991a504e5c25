"""bjxa(1) over this library (bjxa_amd/bjxa, bjxa_amd/csrc/bjxa_cli.c): the
reference's CLI tests restated -- test/test_bjxa.sh (actions, arguments,
messages), test/test_decode.sh (fixture WAV SHA-1s, the saturation vector)
and test/test_decode_error.sh (header and profile errors) -- plus encode
against the survey's reference-encoder SHA-1s.  Both call shapes (one call
per stream, BJXA_CLI_BLOCKS=1 one call per block) must give the same bytes.

The decode/encode checks run on two routes: with no GPU visible (every
call on the library's CPU core) and, under -m gpu, with the offload
threshold at 0 (every call on the HIP kernels).  On failure the output
must be the reference's default per-block loop's: the WAV header plus the
PCM of every whole block before a truncation or a bad block.
"""
import hashlib
import os
import subprocess

import pytest

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
BJXA = os.path.join(ROOT, "bjxa_amd", "bjxa")
# the test build (make testhooks): the same library with BJXA_TEST_FAULT
BJXA_TH = os.path.join(ROOT, "bjxa_amd", "testhooks", "bjxa")
FIXTURES = ["square-mono-4.xa", "square-mono-6.xa", "square-mono-8.xa",
            "square-stereo-4.xa", "square-stereo-6.xa", "square-stereo-8.xa"]


def run(args, stdin=b"", env=None, cwd=None, exe=BJXA):
    e = dict(os.environ)
    if env:
        e.update(env)
    p = subprocess.run([exe] + args, input=stdin, capture_output=True, env=e,
                       cwd=cwd, timeout=120)
    return p.returncode, p.stdout, p.stderr.decode(errors="replace")


def sha1(b):
    return hashlib.sha1(b).hexdigest()


@pytest.fixture(scope="module")
def cli(built):
    assert os.access(BJXA, os.X_OK), "bjxa not built (make -C bjxa_amd/csrc)"
    return BJXA


def no_gpu():
    return {"HIP_VISIBLE_DEVICES": "-1", "ROCR_VISIBLE_DEVICES": "-1"}


# ---- test/test_bjxa.sh: actions and arguments (no decode needed) ----------

def test_help(cli):
    rc, out, _ = run(["help"], env=no_gpu())
    assert rc == 0 and b"Usage:" in out


@pytest.mark.parametrize("args,msg", [
    ([], "Missing an action"),
    (["unknown"], "Unknown action"),
    (["decode", "src.xa", "dst.wav", "jnk.arg"], "Too many arguments"),
    (["encode", "src.xa", "dst.wav", "jnk.arg"], "Too many arguments"),
    (["encode", "--bits", "4", "src.xa", "dst.wav", "jnk.arg"], "Too many arguments"),
    (["encode", "--bits"], "Missing number of bits per sample"),
    (["encode", "--bits", "5"], "Invalid number of bits per sample"),
    (["encode", "--bits", "8001"], "Invalid number of bits per sample"),
])
def test_usage_errors(cli, args, msg):
    rc, _, err = run(args, env=no_gpu())
    assert rc != 0 and msg in err and "Usage:" in err


@pytest.mark.parametrize("args", [
    ["decode", "{w}/nonexistent.xa"],
    ["decode", "{f}", "{w}/nonexistent/out.wav"],
    ["encode", "{w}/nonexistent.xa"],
    ["encode", "{f}", "{w}/nonexistent/out.xa"],
    ["encode", "--bits", "6", "{w}/nonexistent.xa"],
    ["encode", "--bits", "8", "{f}", "{w}/nonexistent/out.xa"],
])
def test_file_errors(cli, tmp_path, golden, args):
    f = tmp_path / "square-stereo-8.xa"
    f.write_bytes(golden("square-stereo-8.xa"))
    args = [a.format(w=tmp_path, f=f) for a in args]
    rc, _, err = run(args, env=no_gpu())
    assert rc != 0 and "Error:" in err


# ---- test/test_decode_error.sh: header errors (host-side) -----------------

def test_empty_input(cli):
    rc, _, err = run(["decode"], b"", env=no_gpu())
    assert rc != 0 and "bjxa_fread_header" in err


def test_header_errors(cli, manifest):
    n = 0
    for v in manifest["header_errors"]:
        if v["fails_in"] != "bjxa_fread_header":
            continue
        rc, _, err = run(["decode"], bytes.fromhex(v["hex"]), env=no_gpu())
        assert rc != 0 and "bjxa_fread_header" in err, v["title"]
        n += 1
    assert n == 9


# ---- decode and encode output, CPU core and GPU -----------------------------

ROUTES = ["cpu", pytest.param("gpu", marks=pytest.mark.gpu)]


def route_env(route, shape="stream"):
    e = no_gpu() if route == "cpu" else {"BJXA_OFFLOAD_DECODE": "0",
                                          "BJXA_OFFLOAD_ENCODE": "0"}
    if shape == "blocks":
        e["BJXA_CLI_BLOCKS"] = "1"
    return e


def expected_decode(data):
    """`bjxa decode` output of the reference's per-block loop: the RIFF
    header, then the PCM of each whole block read, stopping before a block
    whose gain nibble is >= 5 (oracle restatement)."""
    import numpy as np
    import oracle
    h = oracle.parse_xa_header(data)
    bits, ch = h["bits"], h["channels"]
    bsz = (bits * 4 + 1) * ch
    blocks = h["data_len"] // bsz
    k = min(blocks, (len(data) - 32) // bsz)
    xa = np.frombuffer(data, np.uint8, offset=32, count=k * bsz)
    pcm, _, done, bad = oracle.decode(xa, k, bits, ch, h["state"],
                                      frames=min(k * 32, h["samples"]))
    n = min(done * 64 * ch, h["samples"] * ch * 2)
    return (oracle.riff_header(ch, h["rate"], h["samples"] * ch * 2) +
            pcm.tobytes()[:n], bad >= 0, k < blocks)


@pytest.mark.parametrize("route", ROUTES)
@pytest.mark.parametrize("shape", ["stream", "blocks"])
def test_decode_fixtures(cli, golden, manifest, shape, route):
    env = route_env(route, shape)
    for name in FIXTURES:
        rc, out, err = run(["decode"], golden(name), env=env)
        assert rc == 0, err
        assert sha1(out) == manifest["fixtures"][name]["wav_sha1"], name


@pytest.mark.parametrize("route", ROUTES)
def test_decode_argument_forms(cli, golden, manifest, tmp_path, route):
    """test/test_bjxa.sh:39-58: file, file -, - - <stdin, file file."""
    want = manifest["fixtures"]["square-stereo-8.xa"]["wav_sha1"]
    f = tmp_path / "square-stereo-8.xa"
    f.write_bytes(golden("square-stereo-8.xa"))
    for args, stdin in [(["decode", str(f)], b""), (["decode", str(f), "-"], b""),
                        (["decode", "-", "-"], f.read_bytes())]:
        rc, out, err = run(args, stdin, env=route_env(route))
        assert rc == 0 and sha1(out) == want, (args, err)
    w = tmp_path / "out.wav"
    rc, out, err = run(["decode", str(f), str(w)], env=route_env(route))
    assert rc == 0 and out == b"" and sha1(w.read_bytes()) == want, err


@pytest.mark.parametrize("route", ROUTES)
def test_decode_saturation(cli, manifest, route):
    """test/test_decode.sh:82-122: clamp at both int16 bounds."""
    rc, out, err = run(["decode"], bytes.fromhex(manifest["boundary"]["hex"]),
                       env=route_env(route))
    assert rc == 0 and sha1(out) == manifest["boundary"]["wav_sha1"], err


@pytest.mark.parametrize("route", ROUTES)
@pytest.mark.parametrize("shape", ["stream", "blocks"])
def test_decode_invalid_profiles(cli, manifest, shape, route):
    """test/test_decode_error.sh:221-282, and the bytes written before the
    error: header plus the PCM of the blocks before the bad one."""
    env = route_env(route, shape)
    n = 0
    for v in manifest["header_errors"]:
        if v["fails_in"] != "bjxa_decode":
            continue
        data = bytes.fromhex(v["hex"])
        rc, out, err = run(["decode"], data, env=env)
        assert rc != 0 and "bjxa_decode: Protocol error" in err, v["title"]
        want, bad, _ = expected_decode(data)
        assert bad and out == want, v["title"]
        n += 1
    assert n == 2


@pytest.mark.parametrize("route", ROUTES)
@pytest.mark.parametrize("shape", ["stream", "blocks"])
@pytest.mark.parametrize("name,at", [("square-mono-8.xa", 5000), ("square-stereo-6.xa", 3001),
                                     ("square-stereo-4.xa", 17)])
def test_decode_bad_block_inside(cli, golden, shape, route, name, at):
    """A fixture with one profile byte turned bad (gain 5..15) in the
    middle: the output stops exactly before that eblock in both shapes."""
    data = bytearray(golden(name))
    h = __import__("oracle").parse_xa_header(data)
    bs = h["bits"] * 4 + 1
    off = 32 + at * bs
    data[off] = (5 + at % 11) << 4 | (data[off] & 15)
    rc, out, err = run(["decode"], bytes(data), env=route_env(route, shape))
    assert rc != 0 and "bjxa_decode: Protocol error" in err
    want, bad, _ = expected_decode(bytes(data))
    assert bad and out == want


@pytest.mark.parametrize("route", ROUTES)
@pytest.mark.parametrize("shape", ["stream", "blocks"])
@pytest.mark.parametrize("cut", [1, 100, 33 * 7 + 5, 5000])
def test_decode_truncated_bytes(cli, golden, shape, route, cut):
    """A stream cut short: every whole block read is written, then
    "fread: End of file", as the reference's per-block loop does."""
    data = golden("square-mono-8.xa")[:-cut]
    rc, out, err = run(["decode"], data, env=route_env(route, shape))
    assert rc != 0 and "fread: End of file" in err
    want, bad, short = expected_decode(data)
    assert short and not bad and out == want


@pytest.mark.parametrize("route", ROUTES)
@pytest.mark.parametrize("shape", ["stream", "blocks"])
def test_encode_fixtures(cli, golden, manifest, shape, route):
    env = route_env(route, shape)
    for wav, by_bits in manifest["encode"].items():
        for bits, want in by_bits.items():
            rc, out, err = run(["encode", "--bits", bits], golden(wav), env=env)
            assert rc == 0 and sha1(out) == want, (wav, bits, err)
    # default: 6 bits
    rc, out, err = run(["encode"], golden("square-stereo.wav"), env=env)
    assert rc == 0 and sha1(out) == manifest["encode"]["square-stereo.wav"]["6"]


@pytest.mark.parametrize("route", ROUTES)
@pytest.mark.parametrize("shape", ["stream", "blocks"])
@pytest.mark.parametrize("cut", [1, 128 * 3 + 7, 100000])
def test_encode_truncated(cli, golden, shape, route, cut):
    """PCM cut short: the XA of every block whose PCM was complete, then
    "fread: End of file" (src/bjxa_encode.c:130-140)."""
    import numpy as np
    import oracle
    wav = golden("square-stereo.wav")
    rc, out, err = run(["encode", "--bits", "4"], wav[:-cut], env=route_env(route, shape))
    assert rc != 0 and "fread: End of file" in err
    data_len = len(wav) - 44
    k = (data_len - cut) // 128
    pcm = np.frombuffer(wav, "<i2", offset=44, count=k * 64).astype(np.int16)
    want = oracle.encode(pcm, k * 32, 4, 2).tobytes()
    assert out[:32].startswith(b"KWD1") and out[32:] == want


def test_sub_block_stream(cli):
    """A stream shorter than one block decodes and encodes in both shapes
    (the per-block loop passes a whole block's buffer)."""
    import oracle
    import numpy as np
    for shape in ("stream", "blocks"):
        env = route_env("cpu", shape)
        pcm = (np.arange(20 * 2, dtype=np.int16) * 997).astype(np.int16)
        wav = oracle.riff_header(2, 8000, pcm.nbytes) + pcm.tobytes()
        rc, xa, err = run(["encode", "--bits", "8"], wav, env=env)
        assert rc == 0, err
        assert xa[32:] == oracle.encode(pcm, 20, 8, 2).tobytes()
        rc, out, err = run(["decode"], xa, env=env)
        assert rc == 0, err
        want, _, _ = expected_decode(xa)
        assert out == want


@pytest.mark.parametrize("route", ROUTES)
@pytest.mark.parametrize("shape", ["stream", "blocks"])
def test_decode_device_failure_writes_no_pcm(cli, golden, shape, route):
    """A decode call that fails for any reason other than a bad profile
    (here EIO, injected by BJXA_TEST_FAULT on every call the offload
    threshold sends to the device -- a hook only the test build has) leaves
    nothing decoded in the buffer: the CLI writes the RIFF header and no
    PCM, then the error (never PCM of a failed call)."""
    assert os.access(BJXA_TH, os.X_OK), "test build missing (make -C bjxa_amd/csrc testhooks)"
    data = golden("square-stereo-8.xa")
    env = route_env(route, shape)
    env["BJXA_TEST_FAULT"] = "gpu-decode"
    if route == "cpu":
        env["BJXA_OFFLOAD_DECODE"] = "1"
    rc, out, err = run(["decode"], data, env=env, exe=BJXA_TH)
    assert rc != 0 and "bjxa_decode: Input/output error" in err
    want, _, _ = expected_decode(data)
    assert out == want[:44]


def test_shipped_library_has_no_fault_hook(cli, golden):
    """The shipped libbjxa.so.0 ignores BJXA_TEST_FAULT (no
    test hook in the product path): the same call decodes normally."""
    data = golden("square-stereo-8.xa")
    env = dict(no_gpu(), BJXA_TEST_FAULT="gpu-decode", BJXA_OFFLOAD_DECODE="1")
    rc, out, err = run(["decode"], data, env=env)
    assert rc == 0, err
    assert out == expected_decode(data)[0]


@pytest.mark.parametrize("value", ["-1", " 5", "+5", "12x", "99999999999999999999999", ""])
def test_offload_threshold_env_rejects_bad_values(built, value):
    """BJXA_OFFLOAD_DECODE must be a plain decimal block count: a sign,
    blanks, junk or an overflowing value fall back to the default (1024)
    with one warning instead of wrapping to 'never offload'."""
    import subprocess
    import sys
    code = ("import bjxa_amd; print(bjxa_amd.offload_threshold(0), "
            "bjxa_amd.offload_threshold(1))")
    env = dict(os.environ, BJXA_OFFLOAD_DECODE=value, **no_gpu())
    p = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True,
                       env=env, cwd=ROOT, timeout=120)
    assert p.returncode == 0, p.stderr
    assert p.stdout.split() == ["1024", "4096"]
    assert ("ignoring BJXA_OFFLOAD_DECODE" in p.stderr) == (value != "")


def test_offload_threshold_env_accepts_count(built):
    import subprocess
    import sys
    code = "import bjxa_amd; print(bjxa_amd.offload_threshold(0))"
    env = dict(os.environ, BJXA_OFFLOAD_DECODE="77", **no_gpu())
    p = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True,
                       env=env, cwd=ROOT, timeout=120)
    assert p.returncode == 0 and p.stdout.split() == ["77"] and p.stderr == ""
