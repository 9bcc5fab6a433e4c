"""Debug: every codec fixture through rpgpu_uncompress, one subprocess each
(bounded), progress appended to gpurun_out/dbg_uncompress.log."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
G = os.path.join(ROOT, "tests", "golden")
LOG = os.path.join(ROOT, "gpurun_out", "dbg_uncompress.log")

ONE = r'''
import sys, os
sys.path.insert(0, %r)
from redpanda_amd.engine import Engine
from redpanda_amd._lib import RpgpuError
from oracle import oracle as O
codec, path = int(sys.argv[1]), sys.argv[2]
data = open(path, "rb").read()
e = Engine(0)
try:
    got = e.uncompress(codec, data); rc = 0
except RpgpuError as x:
    got, rc = b"", -1
orc, want = O.uncompress(codec, data, max(len(data) * 300, 1 << 20))
if rc == (0 if orc == 0 else -1) and got == want:
    print("OK")
else:
    i = next((k for k in range(min(len(got), len(want))) if got[k] != want[k]), -1)
    bad = sum(1 for k in range(min(len(got), len(want))) if got[k] != want[k])
    print("MISMATCH rc=%%d orc=%%d len=%%d want=%%d first=%%d nbad=%%d got=%%s want=%%s" %% (rc, orc, len(got), len(want), i, bad,
          got[max(i-8,0):i+24].hex(), want[max(i-8,0):i+24].hex()))
''' % ROOT


def main():
    man = json.load(open(os.path.join(G, "manifest.json")))
    names = sys.argv[1:] or [e["name"] for e in man["codecs"]]
    codec = {e["name"]: e["codec"] for e in man["codecs"]}
    with open(LOG, "a") as log:
        for n in names:
            log.write(f"{n} ... ")
            log.flush()
            try:
                r = subprocess.run([sys.executable, "-c", ONE, str(codec[n]), os.path.join(G, "codecs", n + ".bin")],
                                   capture_output=True, text=True, timeout=40)
                log.write((r.stdout.strip() or r.stderr.strip()[-300:]) + "\n")
            except subprocess.TimeoutExpired:
                log.write("TIMEOUT\n")
                log.flush()
                return 1
            log.flush()
    return 0


if __name__ == "__main__":
    sys.exit(main())
