import csv, glob, sys, re, collections
for d in sorted(glob.glob(sys.argv[1] + "_p*")):
    for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
        agg = collections.defaultdict(lambda: collections.defaultdict(list))
        for row in csv.DictReader(open(f)):
            k = re.sub(r"\(.*", "", row["Kernel_Name"])[:90]
            agg[k][row["Counter_Name"]].append(float(row["Counter_Value"]))
        for k, cs in agg.items():
            print(d.split("/")[-1], k, {c: round(sum(v) / len(v), 1) for c, v in cs.items()})
