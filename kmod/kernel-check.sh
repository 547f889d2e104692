#!/bin/sh
# kernel-check.sh — verify the kernel interfaces nvme-strom relies on, against
# a kernel source tree and (optionally) its build directory.
#
# The reference refreshed vendored private headers from the RHEL kernel SRPM
# (utils/rhel7-kernel-check.sh).  This provider vendors no private layout; it
# declares ONE private prototype (nvme_init_request) and uses exported
# symbols.  This script checks, for the kernel about to be built against:
#   1. every symbol the module calls is exported (Module.symvers of KDIR);
#   2. nvme_init_request() still has the signature strom_kmod.h declares;
#   3. rq_end_io_fn still takes (struct request *, blk_status_t);
#   4. the namespace ioctl still answers NVME_IOCTL_ID;
#   5. the version gates match the tree (MODULE_IMPORT_NS form,
#      bdev_file_open_by_dev, fd_file).
# Usage: kmod/kernel-check.sh KSRC [KDIR]      exit 0 = all checks passed
set -u
KSRC=${1:?usage: kernel-check.sh KSRC [KDIR]}
KDIR=${2:-$KSRC}
fail=0
ok()  { printf 'ok    %s\n' "$1"; }
bad() { printf 'FAIL  %s\n' "$1"; fail=1; }
has() { grep -Eq "$2" "$KSRC/$1" 2>/dev/null; }

# 1. exported symbols
SYMS="nvme_init_request bmap blk_mq_alloc_request blk_execute_rq_nowait blk_status_to_errno
bdev_start_io_acct bdev_end_io_acct dma_buf_get dma_buf_put dma_buf_dynamic_attach
dma_buf_detach dma_buf_pin dma_buf_unpin dma_buf_map_attachment dma_buf_unmap_attachment
dma_pool_create dma_pool_destroy dma_pool_alloc dma_pool_free filemap_get_folio
filemap_write_and_wait_range kernel_read anon_inode_getfd bus_find_device_by_name
device_find_child_by_name pci_bus_type misc_register proc_create dma_resv_lock
dma_resv_unlock"
if [ -f "$KDIR/Module.symvers" ]; then
  for s in $SYMS; do
    # filemap_get_folio / dma_resv_lock are inline wrappers of exported helpers
    case $s in
      filemap_get_folio) s2=__filemap_get_folio ;;
      dma_resv_lock) s2=dma_resv_lock ;;
      dma_resv_unlock) s2=dma_resv_reset_max_fences ;;
      *) s2=$s ;;
    esac
    if grep -Eq "[[:space:]]$s2[[:space:]]" "$KDIR/Module.symvers"; then ok "export $s2"
    else bad "export $s2 missing from $KDIR/Module.symvers"; fi
  done
else
  echo "skip  exported-symbol check ($KDIR/Module.symvers not found)"
fi

# 2. nvme_init_request signature + export
if has drivers/nvme/host/nvme.h 'void nvme_init_request\(struct request \*req, struct nvme_command \*cmd\)'; then
  ok "nvme_init_request(struct request *, struct nvme_command *)"
else bad "nvme_init_request prototype changed (drivers/nvme/host/nvme.h)"; fi
has drivers/nvme/host/core.c 'EXPORT_SYMBOL_GPL\(nvme_init_request\)' && ok "nvme_init_request exported" \
  || bad "nvme_init_request not exported (drivers/nvme/host/core.c)"

# 3. end_io signature
if has include/linux/blk-mq.h 'typedef enum rq_end_io_ret \(rq_end_io_fn\)\(struct request \*, *blk_status_t\)'; then
  ok "rq_end_io_fn(struct request *, blk_status_t)"
else bad "rq_end_io_fn signature changed (include/linux/blk-mq.h): update strom_end_io"; fi

# 4. NVME_IOCTL_ID on the namespace disk
has drivers/nvme/host/ioctl.c 'case NVME_IOCTL_ID' && ok "NVME_IOCTL_ID handled" \
  || bad "NVME_IOCTL_ID no longer handled (drivers/nvme/host/ioctl.c)"

# 5. version-gated interfaces
VER=$(make -s -C "$KSRC" kernelversion 2>/dev/null || echo unknown)
echo "info  kernel $VER"
has include/linux/module.h 'define MODULE_IMPORT_NS\(ns\).*__stringify' \
  && echo "info  MODULE_IMPORT_NS takes an identifier (< 6.13 form)" \
  || echo "info  MODULE_IMPORT_NS takes a string literal (>= 6.13 form)"
has include/linux/blkdev.h 'bdev_file_open_by_dev' && ok "bdev_file_open_by_dev (>= 6.9 path)" \
  || { has include/linux/blkdev.h 'bdev_open_by_dev' && ok "bdev_open_by_dev (6.8 path)" || bad "no bdev open-by-dev API"; }
has include/linux/file.h 'define fd_file' && ok "fd_file() accessor" || echo "info  no fd_file(): < 6.12 fallback used"
exit $fail
