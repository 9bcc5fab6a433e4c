"""Debug: LZ4 / snappy payloads of a generated C2/C5 segment through
rpgpu_uncompress one subprocess each (bounded); progress appended to
gpurun_out/dbg_frames.log.  Usage: dbg_frames.py [c2|c5] [max]"""
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
LOG = os.path.join(ROOT, "gpurun_out", "dbg_frames.log")

ONE = r'''
import sys
sys.path.insert(0, %r)
from redpanda_amd.engine import Engine
from redpanda_amd._lib import RpgpuError
from oracle import oracle as O
codec, path = int(sys.argv[1]), sys.argv[2]
data = open(path, "rb").read()
e = Engine(0)
try:
    got = e.uncompress(codec, data); rc = 0
except RpgpuError:
    got, rc = b"", -1
orc, want = O.uncompress(codec, data, max(len(data) * 300, 1 << 22))
if rc == (0 if orc == 0 else -1) and got == want:
    print("OK", len(want))
else:
    i = next((k for k in range(min(len(got), len(want))) if got[k] != want[k]), -1)
    print("MISMATCH rc=%%d orc=%%d len=%%d want=%%d first=%%d" %% (rc, orc, len(got), len(want), i))
''' % ROOT


def main():
    import synth
    from oracle import oracle as O
    from redpanda_amd import abi
    which = sys.argv[1] if len(sys.argv) > 1 else "c2"
    mx = int(sys.argv[2]) if len(sys.argv) > 2 else 40
    kw = dict(synth.C2, lz4_linked_ppm=300000, lz4_content_checksum_ppm=300000) if which == "c2" else synth.C5
    a = np.zeros(12 << 20, np.uint8)
    synth.gen_segment(a, 0, **kw)
    r = O.run_job(a, [0, a.size], abi.JOB_CRC)
    b = r.batches
    os.makedirs("/tmp/frames", exist_ok=True)
    with open(LOG, "a") as log:
        k = 0
        for i in range(len(b)):
            codec = int(b["attrs"][i]) & 7
            if codec == 0 or not (b["flags"][i] & abi.F_COMPLETE):
                continue
            p, sz = int(b["file_pos"][i]), int(b["size_bytes"][i])
            pay = bytes(a[p + 61:p + sz])
            path = f"/tmp/frames/f{i}.bin"
            open(path, "wb").write(pay)
            flg = pay[4] if codec == 3 and len(pay) > 5 else 0
            log.write(f"batch {i} codec {codec} flg {flg:#x} n {len(pay)} ... ")
            log.flush()
            try:
                rr = subprocess.run([sys.executable, "-c", ONE, str(codec), path], capture_output=True, text=True,
                                    timeout=30)
                log.write((rr.stdout.strip() or rr.stderr.strip()[-300:]) + "\n")
            except subprocess.TimeoutExpired:
                log.write("TIMEOUT\n")
                return 1
            log.flush()
            k += 1
            if k >= mx:
                break
    return 0


if __name__ == "__main__":
    sys.exit(main())
