"""The patch kernel's HU normalisation divides by 1000 as q0 = x * (1/1000.f);
q = fma(fma(-q0, 1000, x), 1/1000.f, q0) (patch.hip `div1000`).  IEEE single mul / fma round the
same on the host (C fmaf) as v_mul_f32 / v_fma_f32 on gfx950, so this checks on the CPU that the
shortcut equals x / 1000.f bit for bit for every clamped int16 input (ct_clip/data.py:150-152)."""
import os
import shutil
import subprocess
import tempfile

import pytest

SRC = r'''
#include <stdio.h>
#include <math.h>
#include <string.h>
int main(void) {
  const float R = 1.0f / 1000.0f;
  int bad = 0;
  for (int i = -1000; i <= 1000; ++i) {
    volatile float x = (float)i;
    float ref = x / 1000.0f;
    float q0 = x * R;
    float r = fmaf(-q0, 1000.0f, x);
    float q = fmaf(r, R, q0);
    if (memcmp(&q, &ref, 4)) ++bad;
  }
  printf("%d\n", bad);
  return 0;
}
'''


@pytest.mark.skipif(shutil.which('gcc') is None, reason='needs gcc')
def test_div1000_exact_for_every_clamped_hu():
    with tempfile.TemporaryDirectory() as d:
        c, exe = os.path.join(d, 'd.c'), os.path.join(d, 'd')
        with open(c, 'w') as f:
            f.write(SRC)
        subprocess.run(['gcc', '-O2', '-ffp-contract=off', c, '-o', exe, '-lm'], check=True)
        assert subprocess.run([exe], check=True, capture_output=True, text=True).stdout.strip() == '0'
