"""Per-step kernel summary of a rocprofv3 --kernel-trace CSV of bench.py.

Takes the last `nsteps` steps (delimited by the Adam kernel that ends each
step), prints the wall time and busy time (union of kernel intervals) per
step and the kernels by total time per step.
usage: python tools/step_profile.py <kernel_trace.csv> [nsteps=5] [top=30]
"""
import csv, collections, sys
f=sys.argv[1]; nlast=int(sys.argv[2]) if len(sys.argv)>2 else 5
rows=list(csv.DictReader(open(f)))
for r in rows:
    r["s"]=int(r["Start_Timestamp"]); r["e"]=int(r["End_Timestamp"])
    n=r["Kernel_Name"].replace("(anonymous namespace)","anon").split("(")[0]
    r["n"]=n[5:] if n.startswith("void ") else n
rows.sort(key=lambda r:r["s"])
ad=[r["e"] for r in rows if "adam_kernel" in r["n"]]
lo,hi=ad[-nlast-1],ad[-1]
sel=[r for r in rows if lo<r["s"]<=hi]
tot=collections.Counter(); cnt=collections.Counter()
for r in sel:
    tot[r["n"]]+=(r["e"]-r["s"])/1e3; cnt[r["n"]]+=1
print("wall per step %.1f us, kernel-sum %.1f us, launches %.0f"%((hi-lo)/1e3/nlast, sum(tot.values())/nlast, len(sel)/nlast))
# busy time (union of intervals)
iv=sorted((r["s"],r["e"]) for r in sel); busy=0; cs,ce=iv[0]
for s,e in iv[1:]:
    if s>ce: busy+=ce-cs; cs,ce=s,e
    else: ce=max(ce,e)
busy+=ce-cs
print("busy per step %.1f us"%(busy/1e3/nlast))
for k,v in tot.most_common(int(sys.argv[3]) if len(sys.argv)>3 else 30):
    print(f"{v/nlast:8.1f} us/step {cnt[k]/nlast:6.1f} launches {v/cnt[k]:7.1f} us/launch  {k[:80]}")
