"""Per-step kernel times from rocprofv3 --stats CSVs: python tools/kstats.py DIR... [--steps N]"""
import csv
import glob
import sys

argv = sys.argv[1:]
steps = 4
if "--steps" in argv:
    i = argv.index("--steps")
    steps = int(argv[i + 1])
    del argv[i:i + 2]
args = argv
tabs = []
for d in args:
    f = glob.glob(f"{d}/**/*kernel_stats.csv", recursive=True)[0]
    tabs.append({r["Name"]: float(r["TotalDurationNs"]) / 1e6 / steps for r in csv.DictReader(open(f))})
names = sorted(set().union(*tabs), key=lambda n: -max(t.get(n, 0) for t in tabs))
for n in names[:24]:
    short = n.split("(")[0][:58] if not n.startswith("(") else n[:58]
    print(f"{short:58s}" + "".join(f" {t.get(n, 0):8.3f}" for t in tabs))
print(f"{'TOTAL dq::':58s}" + "".join(f" {sum(v for k, v in t.items() if 'dq::' in k):8.3f}" for t in tabs))
