"""Map a profiling round's PMC summary (tools/pmc_summarize.py, kernel template variants) onto the
nature trunk's pass names for bench.py's roofline `traffic`:
  python3 tools/r6/nat_pmc.py gpurun_out/prof_TAG/summary.json > profiles/pmc_hbm_bytes_nature.json
Variants: k_nat_gemm<MODE, LAYER, BN> (fp32 MFMA), k_nat_gemm_bf<MODE, LAYER, BN, TA, NBUF> (bf16
terms), k_nat_conv1_bf; MODE 1 fwd, 2 dX, 3 conv1 dW, 4 dW (nature.hip)."""
import json
import re
import sys

PASS = {(1, 2): 'conv2_fwd', (1, 3): 'conv3_fwd', (2, 3): 'conv3_dx', (2, 2): 'conv2_dx',
        (3, 1): 'conv1_dw', (4, 3): 'conv3_dw', (4, 2): 'conv2_dw', (0, 1): 'conv1_fwd'}


def main(path):
    s = json.load(open(path))
    out = {}
    for name, v in s['kernels'].items():
        n = name.replace(' ', '')
        if n.startswith('k_nat_conv1_bf'):
            key = 'conv1_fwd'
        elif n.startswith('k_nat_conv23<true>'):
            key = 'conv123_fwd'
        elif n.startswith('k_nat_conv23'):
            key = 'conv23_fwd'
        elif n.startswith('k_nat_dx32'):
            key = 'conv32_dx'
        else:
            m = re.match(r'k_nat_gemm(?:_bf)?<(\d+),(\d+),', n)
            if not m:
                continue
            key = PASS.get((int(m.group(1)), int(m.group(2))))
        if key and v.get('hbm_bytes_per_launch') is not None:
            out['nat_' + key] = dict(hbm_bytes=v['hbm_bytes_per_launch'], variant=name,
                                     trace_avg_us=(v.get('trace') or {}).get('avg_us'))
    json.dump(dict(method=s['method'], source=path,
                   hbm_bytes_per_launch={k: v['hbm_bytes'] for k, v in out.items()}, passes=out),
              sys.stdout, indent=1)


if __name__ == '__main__':
    main(sys.argv[1])
