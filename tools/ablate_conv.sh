for S in 512,32,32,64,256,1,1,0 512,32,32,256,64,1,1,0 512,8,8,256,256,3,1,1; do
  for NS in "" "--nostats"; do
    timeout -k 10 60 python tools/conv_one.py --mode fwd --shape $S --cfg 0 $NS | sed "s/^/$NS /" || exit 1
  done
done
