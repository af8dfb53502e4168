# debug: a bucketed context reused across segmented builds (prints, always exits 0)
import os, sys, json
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests"))
from conftest import load_gcz, load_oracle, GOLDEN, case_input
gcz = load_gcz(); oracle = load_oracle()
m = json.load(open(os.path.join(GOLDEN, "manifest.json")))
def run(env, names):
    for k, v in env.items(): os.environ[k] = v
    c = gcz.Context(0)
    for k in env: del os.environ[k]
    for n in names:
        case = m[n]
        kind, payload, L = case_input(case, gcz)
        try:
            info = c.build_fasta_buffered(payload, L, case["buffer"])
            print(env, n, info["layer_size"][:3], "exp", case["expect"]["layer_sizes"][:3],
                  info["layer_size"] == case["expect"]["layer_sizes"], "bucketed", info["bucketed_pairs"], flush=True)
        except gcz.GczError as e:
            print(env, n, "error", e.code, flush=True)
    c.close()
run({"GCZ_BUCKET_MIN": "1"}, ["segbuf/blank_lines_L12_B3", "segbuf/chmpxx_L12_B1", "segbuf/chmpxx_L12_B1"])
run({"GCZ_BUCKET_MIN": "1"}, ["segbuf/chmpxx_L12_B1", "segbuf/blank_lines_L12_B3", "segbuf/chmpxx_L12_B1"])
run({}, ["segbuf/blank_lines_L12_B3", "segbuf/chmpxx_L12_B1"])
run({"GCZ_BUCKET_MIN": "1"}, ["segbuf/chmpxx_L12_B3", "segbuf/chmpxx_L12_B1"])
run({"GCZ_BUCKET_MIN": "1"}, ["corpus/chmpxx" if False else "segbuf/multi_record_L12_B5", "segbuf/chmpxx_L12_B1"])
