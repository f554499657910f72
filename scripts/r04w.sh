set -o pipefail
# smoke() as the driver runs it, then the audio tests (Vorbis codebook bound is host code)
O=gpurun_out/r04w; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_audio.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/audio.log 2>&1 || { tail -20 $O/audio.log; exit 1; }
tail -1 $O/audio.log
