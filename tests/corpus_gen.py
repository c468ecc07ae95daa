"""Seeded synthetic files with planted secrets and near-misses (test helper).

Produces text in the SURVEY.md §8(d) text model (identifiers, CamelCase,
numbers, punctuation, base64-ish blobs, spaces) with planted instances of
builtin-rule secrets, decoys (one char short, EXAMPLE allow-listed), keyword
sprinkles, CRLF lines, non-ASCII runes (é, K U+212A, ſ U+017F, İ U+0130) and
invalid UTF-8 bytes.
"""
from __future__ import annotations

import random
import string

ALNUM = string.ascii_letters + string.digits
HEX = "0123456789abcdef"
B64 = ALNUM + "+/="


def _r(rng, alphabet, n):
    return "".join(rng.choice(alphabet) for _ in range(n))


def secret_instances(rng):
    """One planted line per template; each matches a builtin rule."""
    up = string.ascii_uppercase + string.digits
    t = [
        lambda: f"AWS_ACCESS_KEY_ID={rng.choice(['AKIA','ASIA','AGPA','A3TX'])}{_r(rng, up, 16)}",
        lambda: f'aws_secret_access_key = "{_r(rng, ALNUM + "/+=", 40)}"',
        lambda: f"  AWS_SECRET_KEY: {_r(rng, ALNUM, 40)}",
        lambda: f"token: ghp_{_r(rng, ALNUM, 36)}",
        lambda: f"gho_{_r(rng, ALNUM, 36)}",
        lambda: f"{rng.choice(['ghu','ghs'])}_{_r(rng, ALNUM, 36)}",
        lambda: f"ghr_{_r(rng, ALNUM, 76)}",
        lambda: f"GITHUB_TOKEN=github_pat_{_r(rng, ALNUM, 22)}_{_r(rng, ALNUM, 59)}",
        lambda: f"glpat-{_r(rng, ALNUM + '-_', 20)}",
        lambda: f"HF_TOKEN=hf_{_r(rng, ALNUM, 39)}",
        lambda: "-----BEGIN RSA PRIVATE KEY-----\n" + "\n".join(_r(rng, B64, 64) for _ in range(rng.randint(1, 4)))
        + "\n-----END RSA PRIVATE KEY-----",
        lambda: f"shp{rng.choice(['ss','at','ca','pa'])}_{_r(rng, HEX, 32)}",
        lambda: f"xox{rng.choice('baprs')}-{_r(rng, ALNUM, rng.randint(10, 48))}",
        lambda: f"{rng.choice(['sk','pk'])}_{rng.choice(['test','live'])}_{_r(rng, string.ascii_lowercase + string.digits, rng.randint(10, 32))}",
        lambda: f"pypi-AgEIcHlwaS5vcmc{_r(rng, ALNUM + '-_', rng.randint(50, 120))}",
        lambda: '  "type": "service_account",',
        lambda: f' heroku_api_key = "{_r(rng, "0123456789ABCDEF", 8)}-{_r(rng, "0123456789ABCDEF", 4)}-{_r(rng, "0123456789ABCDEF", 4)}-{_r(rng, "0123456789ABCDEF", 4)}-{_r(rng, "0123456789ABCDEF", 12)}"',
        lambda: f"https://hooks.slack.com/services/{_r(rng, ALNUM + '+/', rng.randint(44, 48))}",
        lambda: f"SK{_r(rng, HEX, 32)}",
        lambda: f"AGE-SECRET-KEY-1{_r(rng, 'QPZRY9X8GF2TVDW0S3JN54KHCE6MUA7L', 58)}",
        lambda: f'facebook_secret = "{_r(rng, HEX, 32)}"',
        lambda: f'twitter_api_secret: "{_r(rng, HEX, rng.randint(35, 44))}"',
        lambda: f'adobe_client_id = "{_r(rng, HEX, 32)}"',
        lambda: f"p8e-{_r(rng, ALNUM, 32)}",
        lambda: f" LTAI{_r(rng, ALNUM, 20)} ",
        lambda: f"alibaba_secret = '{_r(rng, string.ascii_lowercase + string.digits, 30)}'",
        lambda: f'asana_client_id = "{_r(rng, string.digits, 16)}"',
        lambda: f'atlassian_token := "{_r(rng, string.ascii_lowercase + string.digits, 24)}"',
        lambda: f'bitbucket_key = "{_r(rng, string.ascii_lowercase + string.digits, 32)}"',
        lambda: f'beamer_token = "b_{_r(rng, string.ascii_lowercase + string.digits + "=_-", 44)}"',
        lambda: f"CLOJARS_{_r(rng, ALNUM, 60)}",
        lambda: f"dapi{_r(rng, 'abcdefgh0123456789', 32)}",
        lambda: f'discord_token = "{_r(rng, "abcdefgh0123456789", 64)}"',
        lambda: f'"dp.pt.{_r(rng, ALNUM, 43)}"',
        lambda: f'dropbox_key = "{_r(rng, string.ascii_lowercase + string.digits, 15)}"',
        lambda: f'"duffel_{rng.choice(["test","live"])}_{_r(rng, ALNUM + "_-", 43)}"',
        lambda: f'"dt0c01.{_r(rng, ALNUM, 24)}.{_r(rng, ALNUM, 64)}"',
        lambda: f'"EZ{rng.choice("AT")}K{_r(rng, ALNUM, 54)}"',
        lambda: f'fastly_api = "{_r(rng, string.ascii_lowercase + string.digits, 32)}"',
        lambda: f"FLWSECK_TEST-{_r(rng, 'abcdefgh0123456789', 32)}-X",
        lambda: f"fio-u-{_r(rng, ALNUM + '-_=', 64)}",
        lambda: f'"live_{_r(rng, ALNUM + "-_=", 40)}"',
        lambda: f'"eyJrIjoi{_r(rng, ALNUM + "-_=", 80)}"',
        lambda: f'"{_r(rng, ALNUM, 14)}.atlasv1.{_r(rng, ALNUM + "-_=", 64)}"',
        lambda: f'hubspot_key = "{_r(rng, "abcdefgh0123456789", 8)}-{_r(rng, "abcdefgh0123456789", 4)}-{_r(rng, "abcdefgh0123456789", 4)}-{_r(rng, "abcdefgh0123456789", 4)}-{_r(rng, "abcdefgh0123456789", 12)}"',
        lambda: f'ionic_key = "ion_{_r(rng, string.ascii_lowercase + string.digits, 42)}"',
        lambda: f"jwt = ey{_r(rng, ALNUM, 20)}.ey{_r(rng, ALNUM + '/_-', 25)}.{_r(rng, ALNUM + '/_-', 30)}",
        lambda: f"lin_api_{_r(rng, ALNUM, 40)}",
        lambda: f'lob_key = "{rng.choice(["live","test"])}_{_r(rng, HEX, 35)}"',
        lambda: f'mailgun_key = "key-{_r(rng, HEX, 32)}"',
        lambda: f"pk.{_r(rng, ALNUM, 60)}.{_r(rng, ALNUM, 22)}",
        lambda: f'"NRAK-{_r(rng, up, 27)}"',
        lambda: f'"npm_{_r(rng, ALNUM, 36)}"',
        lambda: f"pscale_pw_{_r(rng, ALNUM + '-_.', 43)}",
        lambda: f"PMAK-{_r(rng, HEX, 24)}-{_r(rng, HEX, 34)}",
        lambda: f"pul-{_r(rng, HEX, 40)}",
        lambda: f"rubygems_{_r(rng, HEX, 48)}",
        lambda: f"SG.{_r(rng, ALNUM + '_-.', 66)}",
        lambda: f"xkeysib-{_r(rng, HEX, 64)}-{_r(rng, ALNUM, 16)}",
        lambda: f"shippo_{rng.choice(['live','test'])}_{_r(rng, HEX, 40)}",
        lambda: f'linkedin_secret = "{_r(rng, string.ascii_lowercase, 16)}"',
        lambda: f'twitch_token = "{_r(rng, string.ascii_lowercase + string.digits, 30)}"',
        lambda: f"typeform_key = tfp_{_r(rng, ALNUM + '-_.=', 59)}",
        lambda: f"  .dockerconfigjson: ey{_r(rng, ALNUM + '/+=', 30)}",
        lambda: f'mailchimp_key = "{_r(rng, HEX, 32)}-us20"',
        lambda: f'messagebird_key = "{_r(rng, string.ascii_lowercase + string.digits, 25)}"',
        lambda: f'newrelic_key = "{_r(rng, up, 64)}"',
        lambda: f'intercom_token = "{_r(rng, string.ascii_lowercase + string.digits + "=_", 60)}"',
    ]
    return t


def noise_line(rng):
    toks = []
    n = rng.randint(2, 14)
    for _ in range(n):
        k = rng.random()
        if k < 0.45:
            toks.append(_r(rng, string.ascii_lowercase + "_", rng.randint(2, 14)))
        elif k < 0.55:
            w = _r(rng, string.ascii_lowercase, rng.randint(2, 8))
            toks.append(w.capitalize() if rng.random() < 0.5 else w.upper())
        elif k < 0.65:
            toks.append(str(rng.randint(0, 10 ** rng.randint(1, 8))))
        elif k < 0.80:
            toks.append(rng.choice(list('=:"\'{}[](),.;')))
        elif k < 0.90:
            toks.append(_r(rng, B64, rng.randint(16, 80)))
        else:
            toks.append(rng.choice([" ", "\t", "  "]))
    return " ".join(toks)


KEYWORD_SPRINKLE = ["key", "aws", "jwt", "sk", "lob", "hf_", "-----", "secret", "token", "dockerc",
                    "heroku", "example", "EXAMPLE", "ghp_", "AKIA", "eyJ", "pk.", "SG.", "live_", "SK"]


def make_file(rng, n_lines=None, secrets=True):
    """Return bytes of one synthetic file."""
    templates = secret_instances(rng)
    lines = []
    n_lines = n_lines if n_lines is not None else rng.randint(0, 60)
    for _ in range(n_lines):
        x = rng.random()
        if secrets and x < 0.08:
            s = rng.choice(templates)()
            y = rng.random()
            if y < 0.1:
                s = s[:-1]  # near miss: one char short
            elif y < 0.15:
                s = s + "EXAMPLE"  # allow-listed by (?i)example
            elif y < 0.25:
                s = noise_line(rng) + " " + s + " " + noise_line(rng)
            lines.append(s)
        elif x < 0.13:
            lines.append(noise_line(rng) + " " + rng.choice(KEYWORD_SPRINKLE) + rng.choice(["", "=", ": ", "_"]) + noise_line(rng))
        else:
            lines.append(noise_line(rng))
    text = "\n".join(lines)
    if rng.random() < 0.5:
        text += "\n"
    data = text.encode()
    r = rng.random()
    if r < 0.05:
        # non-ASCII runes, incl. fold-special ones
        ins = rng.choice(["é", "K", "ſ", "İ", "日本", "Key"]).encode()
        p = rng.randint(0, len(data))
        data = data[:p] + ins + data[p:]
    elif r < 0.08:
        p = rng.randint(0, len(data))
        data = data[:p] + bytes([rng.randint(0x80, 0xFF)]) + data[p:]
    return data


def make_corpus(seed, n_files, secrets=True):
    rng = random.Random(seed)
    files = []
    for i in range(n_files):
        ext = rng.choice(["go", "py", "js", "ts", "yaml", "json", "env", "sh", "txt"])
        path = f"src{rng.randint(0, 99):02d}/pkg{rng.randint(0, 999):03d}/file{i:06d}.{ext}"
        files.append((path, make_file(rng, secrets=secrets)))
    return files
