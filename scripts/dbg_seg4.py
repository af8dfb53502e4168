# debug: repeat the failing sequence under variations (prints, always exits 0)
import os, sys, json, time
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests"))
from conftest import load_gcz, GOLDEN
import numpy as np
gcz = load_gcz()
blank = open(os.path.join(GOLDEN, "fasta", "blank_lines.fa"), "rb").read()
chm = open(os.path.join(GOLDEN, "data", "chmpxx"), "rb").read()
def seq(tag, env, first, dev=False, pause=0.0, reps=4):
    res = []
    for _ in range(reps):
        for k, v in env.items(): os.environ[k] = v
        c = gcz.Context(0)
        for k in env: del os.environ[k]
        try:
            if first is not None:
                c.build_fasta_buffered(first[0], 12, first[1])
            if pause:
                c.sync(); time.sleep(pause)
            if dev:
                buf = c.upload(np.frombuffer(chm, dtype=np.uint8))
                c.sync()
                info = c.build_device_fasta_buffered(buf.ptr, len(chm), 12, 1)
                buf.free()
            else:
                info = c.build_fasta_buffered(chm, 12, 1)
            res.append(info["layer_size"][0])
        except gcz.GczError as e:
            res.append(("err", e.code, e.info["error_offset"]))
        c.close()
    print(tag, res, flush=True)
seq("A", {}, (blank, 3))
seq("A-nograph", {"GCZ_GRAPH": "0"}, (blank, 3))
seq("A-nofused", {"GCZ_FUSED": "0"}, (blank, 3))
seq("A-blankglobal", {}, (blank, 1000))
seq("A-pause", {}, (blank, 3), pause=0.5)
seq("A-dev", {}, (blank, 3), dev=True)
seq("none", {}, None)
seq("A-chm1000first", {}, (chm, 1000))
