"""Print a rocprofv3 *_kernel_stats.csv as short kernel name / calls / average microseconds."""
import csv
import sys

for row in list(csv.reader(open(sys.argv[1])))[1:]:
    n = row[0]
    name = n.split('::')[1].split('(')[0] if '::' in n else n[:40]
    for tag in ('<true>', '<false>', '<0>', '<1>'):
        if tag in n and tag not in name:
            name += tag
    print(f"{name[:44]:44s} calls={row[1]:>5s} avg_us={float(row[3]) / 1e3:8.2f}")
