# Diagnosis: the C++ mirror test binary started from Python (as pytest does) vs from bash.
D=gpurun_out/${1:-r2c_cpp5}
mkdir -p $D
timeout -k 5 100 python -c "
import subprocess, time
t = time.time()
r = subprocess.run(['./mqtt-server_amd/build/test_topics_index'], capture_output=True, text=True, timeout=90)
print('from python: rc', r.returncode, round(time.time() - t, 1), 's'); print(r.stderr[-300:]); print(r.stdout[-200:])
" > $D/py.log 2>&1; echo "py rc=$?"; cat $D/py.log
