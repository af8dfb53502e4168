import csv,sys,re
rows=list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r:int(r["Start_Timestamp"]))
idx=[i for i,r in enumerate(rows) if 'k_mm_init' in r['Kernel_Name']]
i0=idx[-1]
t0=int(rows[i0]["Start_Timestamp"])
for r in rows[i0:]:
    n=re.sub(r"\(anonymous namespace\)::","",r['Kernel_Name'])[:60]
    s=int(r["Start_Timestamp"]); e=int(r["End_Timestamp"])
    if 'k_expand' in n: continue
    print(f"{(s-t0)/1e3:9.1f} {(e-s)/1e3:8.1f}  {n}")
