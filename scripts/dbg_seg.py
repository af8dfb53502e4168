# debug: segmented reader builds under the bucketed node insert (prints, always exits 0)
import os, sys, json
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests"))
from conftest import load_gcz, load_oracle, GOLDEN
gcz = load_gcz(); oracle = load_oracle()
data = open(os.path.join(GOLDEN, "data", "chmpxx"), "rb").read()
envs = [{}, {"GCZ_BUCKET_MIN": "1"}, {"GCZ_BUCKET_MIN": "1", "GCZ_BUCKET_TWO": "0"},
        {"GCZ_BUCKET_MIN": "1", "GCZ_PREDUP": "2"}, {"GCZ_BUCKET_MIN": "1", "GCZ_TAIL": "0"}]
for B in (1, 3, 1000):
    o = oracle.build_fasta_buffered(data, 12, B)
    print("B", B, "oracle", o.layer_sizes()[:4], flush=True)
    for env in envs:
        for k, v in env.items(): os.environ[k] = v
        c = gcz.Context(0)
        for k in env: del os.environ[k]
        info = c.build_fasta_buffered(data, 12, B)
        t = c.tree()
        print("  ", env, info["layer_size"][:4], "attempts", info["attempts"], "bucketed", info["bucketed_pairs"],
              "hashed", info["hashed_pairs"], "leaves_ok", t.leaves_bin() == o.leaves_bin(),
              "layers_ok", t.layers_bin() == o.layers_bin(), flush=True)
        c.close()
# global bucketed reference point
os.environ["GCZ_BUCKET_MIN"] = "1"
c = gcz.Context(0)
del os.environ["GCZ_BUCKET_MIN"]
info = c.build_fasta(data, 12)
print("global bucketed", info["layer_size"][:4], info["bucketed_pairs"], flush=True)
