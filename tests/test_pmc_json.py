"""tools/pmc_json.py, which turns one FETCH_SIZE and one WRITE_SIZE
rocprofv3 capture into the traffic JSON bench.py reports (roofline.traffic):
units (KiB), the gfx950 FETCH_SIZE doubling, per-dispatch means, and the
bench's own reader (bench.pmc_traffic) on the result."""
import csv
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _capture(path, counter, rows):
    with open(path, 'w', newline='') as f:
        w = csv.DictWriter(f, fieldnames=['Dispatch_Id', 'Kernel_Name', 'Counter_Name', 'Counter_Value',
                                          'Start_Timestamp', 'End_Timestamp'])
        w.writeheader()
        for d, (k, v, ns) in enumerate(rows):
            w.writerow({'Dispatch_Id': d, 'Kernel_Name': k, 'Counter_Name': counter, 'Counter_Value': v,
                        'Start_Timestamp': 1000, 'End_Timestamp': 1000 + ns})


def test_pmc_json(tmp_path):
    demod = 'void aero::demod_oqpsk_kernel<false>(aero::DevState, aero::DevTables, int, int)'
    coarse = 'void aero::coarse_kernel<0>(aero::DevState, aero::DevTables, int)'
    f, w, out = tmp_path / 'f.csv', tmp_path / 'w.csv', tmp_path / 'pmc.json'
    _capture(f, 'FETCH_SIZE', [(demod, 1000.0, 10), (demod, 3000.0, 30), (coarse, 500.0, 7)])
    _capture(w, 'WRITE_SIZE', [(demod, 4000.0, 20), (demod, 4000.0, 20), (coarse, 100.0, 7)])
    subprocess.run([sys.executable, os.path.join(ROOT, 'tools', 'pmc_json.py'), str(f), str(w), str(out),
                    'oqpsk10500', '65536', 'test'], check=True, capture_output=True)
    d = json.load(open(out))
    k = d['kernels']['demod_oqpsk_kernel<false>']
    assert k['fetch_bytes_x2'] == 2 * 2000 * 1024          # mean 2000 KiB, doubled
    assert k['write_bytes'] == 4000 * 1024
    assert d['hbm_bytes_per_launch'] == k['fetch_bytes_x2'] + k['write_bytes']
    assert d['algorithmic_bytes_per_launch'] == int(18.22 * 65536 * 4096)
    sys.path.insert(0, ROOT)
    import bench
    assert bench.pmc_traffic(str(out), 'oqpsk10500', 65536, 'demod_oqpsk_kernel')[0] == d['hbm_bytes_per_launch']
    kc = d['kernels']['coarse_kernel<0>']
    assert bench.pmc_traffic(str(out), 'oqpsk10500', 65536, 'coarse_kernel')[0] == kc['hbm_bytes_per_launch']
    assert bench.pmc_traffic(str(out), 'oqpsk10500', 1024, 'coarse_kernel') == (None, None)   # another configuration
    assert bench.pmc_traffic(str(out), 'oqpsk10500', 65536, 'viterbi_kernel') == (None, None)  # not captured
