for r in 16 32 64; do CASK_RUN_CHUNKS=$r CASK_NO_REPAIR=1 timeout -k 10 200 python tools/time_variant.py run$r 2>&1 | grep -v amdgpu.ids || exit 1; done
