R=$(pwd); O=gpurun_out/r4qt; mkdir -p $O
AB_STEPS=500 timeout -k 10 1000 python -u tools/ab.py 3 base: qt32k:LPC_Q_TARGET=32768 qt16k:LPC_Q_TARGET=16384 qt131k:LPC_Q_TARGET=131072 rs16:LPC_ROOTS_S=16 rs4:LPC_ROOTS_S=4 > $O/ab_qt.log 2>&1 || { tail $O/ab_qt.log; exit 1; }
tail -1 $O/ab_qt.log
