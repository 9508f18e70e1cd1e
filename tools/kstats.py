"""Print a rocprofv3 kernel_stats.csv as name / calls / avg us / total us / %."""
import csv
import sys

for r in csv.DictReader(open(sys.argv[1])):
    print(f"{r['Name'][:48]:48s} {int(r['Calls']):6d} {float(r['AverageNs']) / 1e3:9.1f} "
          f"{float(r['TotalDurationNs']) / 1e3:10.1f} {float(r['Percentage']):6.2f}")
