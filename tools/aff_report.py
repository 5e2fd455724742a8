"""Per-dispatch report of the batch-affine level kernels and the G1 accumulation from a
tools/r4_prof.sh output directory: duration, VALU instructions, issue rate."""
import collections
import csv
import sys

d = sys.argv[1]
rows = list(csv.DictReader(open(f"{d}/trace/run_kernel_trace.csv")))
want = lambda n: "k_aff_" in n or "k_accumulate_pf<CurveOps<FpOpsT" in n
sel = [r for r in rows if want(r["Kernel_Name"])]
print("last proof, kernel trace:")
for r in sel[-(len(sel) // 3):]:
    t = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
    print(f"  {r['Kernel_Name'].split('(')[0][-26:]:28s} grid {r['Grid_Size_X']:>8} {t:7.3f} ms")
sq = list(csv.DictReader(open(f"{d}/sq/run_counter_collection.csv")))
per = collections.OrderedDict()
for r in sq:
    e = per.setdefault(r["Dispatch_Id"], {"name": r["Kernel_Name"],
                                          "t": (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6})
    e[r["Counter_Name"]] = float(r["Counter_Value"])
v = [x for x in per.values() if want(x["name"])]
print("SQ pass, last proof:")
for x in v[-(len(v) // 3):]:
    print(f"  {x['name'].split('(')[0][-26:]:28s} {x['t']:7.3f} ms VALU {x['SQ_INSTS_VALU']:.3e} "
          f"{x['SQ_INSTS_VALU'] / x['t'] / 1e6:6.1f} G/s  VMEM_RD {x['SQ_INSTS_VMEM_RD']:.2e}")
