"""Per-kernel averages of one rocprofv3 --pmc pass (run_counter_collection.csv): the quick
check of a counter after a kernel change (tools/gpu_quick.sh, PMC=...)."""
import collections
import csv
import sys


def main():
    path = sys.argv[1]
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for r in csv.DictReader(open(path)):
        k = r["Kernel_Name"].split("(")[0]
        acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[k].add(r["Dispatch_Id"])
    for k in sorted(acc):
        n = len(disp[k])
        print(k, n, {c: round(v / n) for c, v in sorted(acc[k].items())})


if __name__ == "__main__":
    main()
