import sys, ctypes as C, os
sys.path.insert(0,'webp-decoder_amd'); sys.path.insert(0,'.'); sys.argv=['bench.py','--no-cpu-baseline','--steps','1','--warmup','0','--frames','32']
os.environ['VP8G_LIB']='webp-decoder_amd/lib/diag/libvp8g_stamps.so'
import bench, vp8g
bench.main()
lib=vp8g.gpu_lib()
a=(C.c_ulonglong*64)(); lib.vp8g_debug_wave_times(a)
b=(C.c_ulonglong*16)(); lib.vp8g_debug_stamps(b,0)
t0=min(a[i] for i in range(0,64,2) if a[i])
for w in range(8): print('wave',w,'start us',(a[2*w]-t0)/100,'end us',(a[2*w+1]-t0)/100)
print('memtime', b[8], 'realtime', b[9])
