"""Same-box A/B of the bench step under environment settings (each setting its own child
process, interleaved rounds):  python tools/env_ab.py "" "CTCLIP_EPI_LDS=3" ...   (GPU)"""
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    sets = sys.argv[1:] or ['']
    for rnd in range(3):
        for st in sets:
            env = dict(os.environ)
            for kv in st.split():
                k, v = kv.split('=', 1)
                env[k] = v
            r = subprocess.run([sys.executable, '-u', os.path.join(REPO, 'bench.py'), '--steps', '10', '--warmup', '3',
                                '--no-cpu-baseline', '--no-precise'], env=env, capture_output=True, text=True)
            if r.returncode != 0:
                print(r.stdout[-2000:], r.stderr[-2000:])
                sys.exit(r.returncode)
            d = json.loads([x for x in r.stdout.splitlines() if x.startswith('{')][-1])
            print(f"[{st or 'default'}] {d['value']:.2f} pairs/s  {d['ms_per_step']:.3f} ms/step  "
                  f"vit_fwd {d.get('vit_forward', {}).get('ms')}", flush=True)


if __name__ == '__main__':
    main()
