"""Regenerate tests/golden/ from the reference checkout (run in the build
container only; the GPU box never reads /root/reference).

What is here and where it comes from:
  square-{mono,stereo}-{4,6,8}.xa.gz   the reference's own decode fixtures
                                       (test/*.xa), gzip'd byte-for-byte
  square-{mono,stereo}.wav.gz          the reference's PCM fixtures (test/*.wav)
  manifest.json                        expected SHA-1s:
     xa_sha1 / wav_sha1   test/test_decode.sh:24-78 (input file, decoded WAV)
     boundary             test/test_decode.sh:88-122 (hex vector + WAV SHA-1)
     header_errors        test/test_decode_error.sh:32-219 (hex headers)
     encode               SURVEY.md App. B: `bjxa encode --bits N` on the
                          .wav fixtures, from the reference built during the
                          survey (no reference test pins encode output)

Only data (inputs and expected outputs) is copied; no reference source.
"""
import gzip
import json
import os
import re
import shutil

REF = "/root/reference/test"
HERE = os.path.dirname(os.path.abspath(__file__))


def hexblock(text):
    """annotated hex heredoc -> bytes (same rules as test/hex_decode)."""
    out = []
    for line in text.splitlines():
        line = line.split("|")[0].strip()
        if line and not line.startswith("#"):
            out.append(line.replace(" ", ""))
    return bytes.fromhex("".join(out))


def main():
    for name in sorted(os.listdir(REF)):
        if name.endswith((".xa", ".wav")):
            with open(os.path.join(REF, name), "rb") as f, \
                    gzip.open(os.path.join(HERE, name + ".gz"), "wb", 9) as g:
                shutil.copyfileobj(f, g)

    dec = open(os.path.join(REF, "test_decode.sh")).read()
    pairs = re.findall(r'expect_sha1 "([0-9a-f]{40})" \\\n\s*cat <"\$TEST_DIR"/(\S+)\n\s*'
                       r'expect_sha1 "([0-9a-f]{40})"', dec)
    fixtures = {n: {"xa_sha1": a, "wav_sha1": b} for a, n, b in pairs}
    heredocs = re.findall(r"mk_hex <<EOF\n(.*?)\nEOF\n\s*\n?\s*expect_(\w+) \"([^\"]+)\"",
                          dec, re.S)
    boundary = {"hex": hexblock(heredocs[0][0]).hex(), "wav_sha1": heredocs[0][2]}

    err = open(os.path.join(REF, "test_decode_error.sh")).read()
    header_errors = []
    title = None
    lines = err.splitlines()
    i = 0
    while i < len(lines):
        ln = lines[i]
        if ln.startswith("_ ") and not ln.startswith("_ -"):
            title = ln[2:].strip()
        if ln.startswith("mk_hex <<EOF"):
            j = lines.index("EOF", i + 1)
            body = "\n".join(lines[i + 1:j])
            k = j + 1
            while not lines[k].startswith("expect_error"):
                k += 1
            fails_in = re.match(r'expect_error "(\w+)"', lines[k]).group(1)
            header_errors.append({"title": title, "hex": hexblock(body).hex(),
                                  "fails_in": fails_in})
            i = k
        i += 1

    encode = {
        "square-mono.wav": {"4": "422af2b8247caaff011c3a925e7735c4c4e09fc7",
                            "6": "ce97d26d4e0f4a93fbf2883c56a1607ecc543bea",
                            "8": "82d39ab8e3ee1d5832afcff3c9e5bd35b708f014"},
        "square-stereo.wav": {"4": "d525f1818f6913ee408d2dfb194c75cb62010160",
                              "6": "76779e51d6ee5e45ac673bb81751c9f83588e2bf",
                              "8": "1d34cf95cf518dde306175fffded026c1295112f"},
    }
    man = {"fixtures": fixtures, "boundary": boundary,
           "header_errors": header_errors, "encode": encode}
    with open(os.path.join(HERE, "manifest.json"), "w") as f:
        json.dump(man, f, indent=1, sort_keys=True)
    print(len(fixtures), "fixtures,", len(header_errors), "header error vectors")


if __name__ == "__main__":
    main()
