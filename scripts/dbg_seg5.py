# debug: which seg builds fail after an earlier small build (prints, always exits 0)
import os, sys, json
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests"))
from conftest import load_gcz, load_oracle, GOLDEN
gcz = load_gcz(); oracle = load_oracle()
blank = open(os.path.join(GOLDEN, "fasta", "blank_lines.fa"), "rb").read()
chm = open(os.path.join(GOLDEN, "data", "chmpxx"), "rb").read()
def seq(tag, env, steps):
    for k, v in env.items(): os.environ[k] = v
    c = gcz.Context(0)
    for k in env: del os.environ[k]
    res = []
    for data, B in steps:
        try:
            info = c.build_fasta_buffered(data, 12, B)
            o = oracle.build_fasta_buffered(data, 12, B)
            t = c.tree()
            res.append((B, info["layer_size"][0], t.leaves_bin() == o.leaves_bin(), t.layers_bin() == o.layers_bin(), info["attempts"]))
        except gcz.GczError as e:
            res.append((B, "err", e.code, e.info["error_offset"]))
    print(tag, res, flush=True)
    c.close()
seq("fresh B1 x3", {}, [(chm, 1)] * 3)
for B in (1, 2, 3, 5, 7, 1000, 4095):
    seq(f"blank then B{B}", {}, [(blank, 1000), (chm, B)])
seq("blank then B1 notail", {"GCZ_TAIL": "0"}, [(blank, 1000), (chm, 1)])
seq("blank then B1 wide", {"GCZ_TABLE": "wide"}, [(blank, 1000), (chm, 1)])
seq("blank then B1 cap0", {"GCZ_SMALL_CAP_SHIFT": "0"}, [(blank, 1000), (chm, 1)])
seq("blank then B1 leafcap", {"GCZ_SMALL_LEAF_SHIFT": "0"}, [(blank, 1000), (chm, 1)])
seq("chmB1000 then B1", {}, [(chm, 1000), (chm, 1)])
seq("chmB3 then B1", {}, [(chm, 3), (chm, 1)])
