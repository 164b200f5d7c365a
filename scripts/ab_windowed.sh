set -u
O=gpurun_out/win; mkdir -p $O
L=$PWD/gym-sparksched_amd/build/ab/win_nofb.so
SSIM_LIB=$L SSIM_WINDOW=1 timeout -k 10 200 python bench.py --no-cpu-baseline --workload large --steps 100 --warmup 20 > $O/large_win.log 2>&1 || exit $?
timeout -k 10 200 python bench.py --no-cpu-baseline --workload large --steps 100 --warmup 20 > $O/large_main.log 2>&1 || exit $?
SSIM_LIB=$L SSIM_WINDOW=1 timeout -k 10 200 python bench.py --no-cpu-baseline --workload decima --steps 40 --warmup 5 > $O/decima_win.log 2>&1 || exit $?
timeout -k 10 200 python bench.py --no-cpu-baseline --workload decima --steps 40 --warmup 5 > $O/decima_main.log 2>&1 || exit $?
