"""Summarise rocprofv3 --pmc counter_collection.csv files: mean counter value
per dispatch for each engine kernel (used to build profiles/*pmc*.json)."""
import csv
import json
import sys
from collections import defaultdict


def load(paths):
    acc = defaultdict(lambda: defaultdict(list))
    for p in paths:
        for r in csv.DictReader(open(p)):
            k = r['Kernel_Name'].split('(')[0].replace('void ', '').replace('aero::', '')
            acc[k][r['Counter_Name']].append((int(r['Dispatch_Id']), float(r['Counter_Value']),
                                              int(r['End_Timestamp']) - int(r['Start_Timestamp'])))
    return acc


def summary(acc):
    out = {}
    for k, cs in acc.items():
        d = {}
        for cn, v in cs.items():
            d[cn] = sum(x[1] for x in v) / len(v)
            d['dispatches'] = len(v)
            d['avg_ns'] = sum(x[2] for x in v) / len(v)
        out[k] = d
    return out


if __name__ == '__main__':
    print(json.dumps(summary(load(sys.argv[1:])), indent=1))
