set -u
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_audio.py tests/test_gpu_beam.py tests/test_gpu_kernels.py -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread -rA -s > gpurun_out/r06a_gputest.txt 2>&1
rc=$?; tail -3 gpurun_out/r06a_gputest.txt; grep "mp3 vs vorbis" gpurun_out/r06a_gputest.txt
exit $rc
