tools/gpu_steps.sh \
  "300:qt:python tools/quick_time.py 3,256,6,1 3,256,6,1" \
  "300:qts1:GM_LIB_PATH=_exp/libgm_s1.so python tools/quick_time.py 3,256,6,1 3,256,6,1"
