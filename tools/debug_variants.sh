for v in nn_base nn_u2 nn_u4 nn_q2 nn_q2u4 nn_base; do
  RBE_LIB_PATH=build/variants/lib_$v.so timeout -k 10 120 python -u tools/c5_profile.py > gpurun_out/nnv_$v.log 2>&1 || { echo "$v failed"; exit 1; }
  echo "$v: $(grep 'prof=1' gpurun_out/nnv_$v.log | sed 's/.*NN [0-9]* launches \([0-9.]*\) ms.* \([0-9.]*\) TF64.*/\1 ms \2 TF/' | tr '\n' ' ')"
done
