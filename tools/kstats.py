"""Prints the average kernel times of rocprofv3 --stats CSVs: python tools/kstats.py DIR..."""
import csv
import sys

for d in sys.argv[1:]:
    print("==", d)
    for r in csv.DictReader(open(f"{d}/run_kernel_stats.csv")):
        n = r["Name"].replace("fm3d::(anonymous namespace)::", "").replace("void ", "")
        n = n[: n.find("(")] if "(" in n else n
        print(f"  {n[-60:]:62s} {int(r['Calls']):5d} {float(r['AverageNs']) / 1e3:10.1f} us")
