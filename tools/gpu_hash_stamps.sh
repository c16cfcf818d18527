timeout -k 10 60 ./tools/ubench_valu > gpurun_out/ubench_valu.log 2>&1; cat gpurun_out/ubench_valu.log
CASK_FUSE_CHASE=1 CASK_HASH_H0=8 timeout -k 10 200 python tools/hash_stamps.py > gpurun_out/hash_stamps_h8.log 2>&1; tail -8 gpurun_out/hash_stamps_h8.log
CASK_FUSE_CHASE=1 timeout -k 10 200 python tools/hash_stamps.py > gpurun_out/hash_stamps_h16.log 2>&1; tail -8 gpurun_out/hash_stamps_h16.log
timeout -k 10 200 python tools/hash_stamps.py > gpurun_out/hash_stamps_nofuse.log 2>&1; tail -8 gpurun_out/hash_stamps_nofuse.log
