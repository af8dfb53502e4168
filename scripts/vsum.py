import json, sys
tag = sys.argv[1]
for R in (8, 2):
    try:
        d = json.loads(open(f'gpurun_out/strong_{tag}_v{R}.log').read().strip().splitlines()[-1])
    except Exception as e:
        print(R, e); continue
    par = all(v for k, v in (d['parity'] or {}).items() if 'match' in k)
    print(f"R={R} {d['value']/1e9:.1f} Gbase/s {d['ms_per_step']:.3f} ms/step parity {par} rank_kernel_ms {d.get('rank_kernel_ms')}")
    for k, v in d['kernels'].items():
        print(f"    {k:16s} {v['launches']:3d} {v['total_ms']:.4f}")
