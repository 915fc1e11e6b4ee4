cd /root/repo && mkdir -p gpurun_out
for pad in 0 20000 60000; do
GWAMD_POA_LDS_PAD=$pad timeout -k 10 300 python bench.py --steps 2 --no-cpu > gpurun_out/occ_$pad.log 2>&1 || exit 1
done
