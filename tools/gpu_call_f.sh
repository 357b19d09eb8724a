tools/gpu_steps.sh \
  "300:qt:python tools/quick_time.py 3,256,4,1 3,256,6,1 3,256,6,1" \
  "300:qt8:GM_LIB_PATH=_exp/libgm_w8.so python tools/quick_time.py 3,256,6,1 3,256,6,1"
