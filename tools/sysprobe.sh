#!/bin/bash
# Collects host/storage facts on the GPU box (no GPU kernels run).
set -u
out=gpurun_out/sysprobe.txt
{
echo "== uname"; uname -a
echo "== whoami"; id
echo "== nproc"; nproc
echo "== mem"; free -g
echo "== df"; df -hT 2>&1
echo "== mounts"; cat /proc/mounts | head -40
echo "== lsblk"; lsblk -o NAME,SIZE,TYPE,ROTA,MODEL,MOUNTPOINT 2>&1 | head -60
echo "== nvme"; ls -l /dev/nvme* 2>&1 | head; ls /sys/class/nvme 2>&1
echo "== proc nvme-strom"; ls -l /proc/nvme-strom /dev/nvme-strom 2>&1
echo "== kernel build"; ls /lib/modules/$(uname -r)/build 2>&1 | head -3
echo "== numa"; ls /sys/devices/system/node/ 2>&1; cat /sys/devices/system/node/node*/cpulist 2>&1
echo "== rocm-smi"; timeout 60 rocm-smi --showbus --showmeminfo vram 2>&1 | head -30
echo "== gcc probe"; gcc -O2 -o /tmp/sysprobe_$$ tools/sysprobe.c && /tmp/sysprobe_$$ /tmp "$PWD" /dev/shm ${TMPDIR:-/tmp}
echo "== TMPDIR=${TMPDIR:-unset} HOME=$HOME"
echo "== dd direct write+read 2GiB in $PWD"
f=$PWD/gpurun_out/.ddtest
timeout 120 dd if=/dev/urandom of=$f bs=16M count=128 oflag=direct 2>&1 | tail -1
timeout 120 dd if=$f of=/dev/null bs=4M iflag=direct 2>&1 | tail -1
timeout 120 dd if=$f of=/dev/null bs=128k iflag=direct 2>&1 | tail -1
timeout 120 dd if=$f of=/dev/null bs=4k count=50000 iflag=direct 2>&1 | tail -1
rm -f $f
echo "== dd in /tmp"
f=/tmp/.ddtest_$$
timeout 120 dd if=/dev/urandom of=$f bs=16M count=128 oflag=direct 2>&1 | tail -1
timeout 120 dd if=$f of=/dev/null bs=4M iflag=direct 2>&1 | tail -1
rm -f $f
} > $out 2>&1
echo done
