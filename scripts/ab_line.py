"""One bench JSON line (stdin) -> "value ms_per_step kernel=ms ..." for A/B tables."""
import json
import sys

d = json.loads(sys.stdin.read())
ks = ' '.join('%s=%.3f' % (k.replace('_kernel', ''), v['ms_per_step']) for k, v in d.get('kernels', {}).items())
print(d['value'], d['ms_per_step'], ks)
