"""Private-key verify micro bench (TSG_PROFILE_VERIFY): 64 files, one key each;
argv[1] == "example" puts the allow word in every key (the allow VM runs)."""
import os
import sys

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
os.environ["TSG_PROFILE_VERIFY"] = "1"
import trivy_amd.secret as S  # noqa: E402

body = "A" * 64 + "\n" + "B" * 40
if len(sys.argv) > 1 and sys.argv[1] == "example":
    body = "A" * 30 + "EXAMPLE" + "A" * 27 + "\n" + "B" * 40
key = "-----BEGIN RSA PRIVATE KEY-----\n" + body + "\n-----END RSA PRIVATE KEY-----"
files = [(f"f{i}.txt", ("hello world\n" * 50 + key + "\nfoo = bar\n" * 20).encode()) for i in range(64)]
sc = S.new_scanner(None)
for it in range(3):
    got = sc.scan_batch([S.ScanArgs(p, d) for p, d in files])
print(sum(len(g.Findings) for g in got))
