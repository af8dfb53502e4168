# debug: which earlier build breaks a later segmented build (prints, always exits 0)
import os, sys, json
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests"))
from conftest import load_gcz, load_oracle, GOLDEN, case_input
gcz = load_gcz()
m = json.load(open(os.path.join(GOLDEN, "manifest.json")))
blank = open(os.path.join(GOLDEN, "fasta", "blank_lines.fa"), "rb").read()
chm = open(os.path.join(GOLDEN, "data", "chmpxx"), "rb").read()
exp = m["segbuf/chmpxx_L12_B1"]["expect"]["layer_sizes"]
def seq(tag, env, steps):
    for k, v in env.items(): os.environ[k] = v
    c = gcz.Context(0)
    for k in env: del os.environ[k]
    out = []
    for kind, data, B in steps:
        try:
            if kind == "buf":
                info = c.build_fasta_buffered(data, 12, B)
            else:
                info = c.build_fasta(data, 12)
            out.append((kind, B, info["layer_size"][:2], info["attempts"]))
        except gcz.GczError as e:
            out.append((kind, B, "err", e.code, e.info["error_offset"] if e.info else None,
                        e.info["error_symbol"] if e.info else None))
    print(tag, out, "exp", exp[:2], flush=True)
    c.close()
seq("A blank-buf3 chm-buf1", {}, [("buf", blank, 3), ("buf", chm, 1)])
seq("B blank-plain chm-buf1", {}, [("plain", blank, 0), ("buf", chm, 1)])
seq("C blank-buf3 chm-plain", {}, [("buf", blank, 3), ("plain", chm, 0)])
seq("D chm-plain chm-buf1", {}, [("plain", chm, 0), ("buf", chm, 1)])
seq("E blank-buf3 chm-buf1 nograph", {"GCZ_GRAPH": "0", "GCZ_FUSED": "0"}, [("buf", blank, 3), ("buf", chm, 1)])
seq("F blank-buf3 chm-buf1000", {}, [("buf", blank, 3), ("buf", chm, 1000)])
seq("G blank-buf3 chm-buf1 x2", {}, [("buf", blank, 3), ("buf", chm, 1), ("buf", chm, 1)])
seq("H chm-buf1 only", {}, [("buf", chm, 1)])
