"""Inputs of the fold-special cliff cases (tests/test_gpu_fold.py; expected
findings made by tools/make_fold_fixture.py with the CPU oracle into
tests/golden/fold_big.json).  Each case is a 64 MiB file of the bench corpus
(tsg_gen_file host twin, seeded) with a few lines spliced in that spell
keywords / anchor literals with İ (U+0130), K (U+212A) or ſ (U+017F)."""
import ctypes

SECRET40 = "AbCdEfGhIjKlMnOpQrStUvWxYz0123456789+/=A"
CASES = [
    {"name": "one-long-s", "seed": 99, "file": 5, "size": 64 << 20, "density": 1e-5,
     "inserts": [[0.5, "aws_ſecret_access_key = \"" + SECRET40 + "\""]]},
    {"name": "kelvin-and-dotted-i", "seed": 101, "file": 9, "size": 64 << 20, "density": 1e-5,
     "inserts": [[0.25, "aws_secret_access_Key = \"" + SECRET40[::-1] + "\""],
                 [0.5, "lİnkedin_secret = \"abcdefghijklmnop\""],
                 [0.75, "Key: sk_live_0123456789abcdefghij ſk_test_abcdefghij0123456789"]]},
]


def build(N, case):
    """The case's bytes: the generated file with each insert spliced in as its
    own line after the first newline at or past fraction x of the file."""
    n = case["size"]
    buf = (ctypes.c_uint8 * n)()
    N.check(N.gen.tsg_gen_file(case["seed"], case["file"], n, case["density"], buf))
    data = bytes(buf)
    for frac, text in sorted(case["inserts"], key=lambda t: -t[0]):
        p = data.index(b"\n", int(len(data) * frac))
        data = data[:p + 1] + text.encode("utf-8") + b"\n" + data[p + 1:]
    return data
