import json, sys
l = open(sys.argv[1]).read().strip().splitlines()[-1]
d = json.loads(l)
print(round(d['value'] / 1e9, 2), "Gbase/s", round(d['ms_per_step'], 4), "ms/step", "parity", all(v for k, v in (d.get('parity') or {}).items() if k.endswith('match')))
for k, v in d['kernels'].items():
    print(f"  {k:16s} {v['launches']:3d} {v['total_ms']:.4f}")
