/* kshim_sim.h — the harness side of the kernel model (kshim_rt.c): building
 * the simulated machine (controllers, namespaces, md arrays, filesystems,
 * page cache, dma-bufs), opening the module's device, and reading back the
 * contract and leak counters.  Used by kmod_exec.c and, through ctypes, by
 * tests/test_kmod_exec_cpu.py. */
#ifndef KSHIM_SIM_H
#define KSHIM_SIM_H
#include <stdint.h>

#define ENOTTY_SIM 25
#define ENODEV_SIM 19
#define STROM_SIM_MAX_PRPS 1024

/* all int64 so the struct reads as an array (ctypes mirrors the order) */
struct ksim_counters {
	int64_t violations;
	int64_t printk;
	int64_t kmallocs_live;
	int64_t pages_live;
	int64_t iommu_pages_live;
	int64_t requests_live;
	int64_t files_live;
	int64_t module_refs;
	int64_t dmabufs_live;
	int64_t folio_refs;
	int64_t cmds_submitted;
	int64_t cmds_ok;
	int64_t cmds_bad;
	int64_t cmds_failed_injected;
	int64_t bytes_moved;
	int64_t dma_map_calls;
	int64_t writebacks;
	int64_t deferred_fputs;
	int64_t fds_leaked;
	int64_t dev_refs_leaked;
	int64_t iommu_pages_leaked;
};

int ksim_init(void);
void ksim_fini(void);
void ksim_quiesce(void);
int ksim_module_load(void);
void ksim_module_unload(void);
void ksim_counters(struct ksim_counters *out);
const char *ksim_last_violation(void);

void ksim_set_euid(unsigned int uid);
void ksim_set_admin(int on);
void ksim_set_signal(int on);
void ksim_set_verbose(int v);
void ksim_poison_user(const void *p, size_t n);
void ksim_fail_cmd(int nth, int blk_status);
void ksim_fail_map(int nth);
void ksim_dma_max_mapping(size_t bytes);   /* refuse dma_map_page larger than this */

int ksim_ctrl_new(const char *pci_name, int numa_node);
void ksim_ctrl_config(int ctrl, int reorder, int delay_us, int hold);
int ksim_ctrl_queued(int ctrl);
void ksim_ctrl_set_dma_mask_bits(int ctrl, int bits);
int ksim_ns_new(int ctrl, uint32_t nsid, int lba_shift, uint64_t nsects, uint32_t max_hw_sectors,
		int hidden);
int ksim_md_new(const int *members, int n, uint32_t chunk_sects, const uint64_t *data_offset);
int ksim_head_new(int path_disk);
uint32_t ksim_disk_devt(int disk);
const char *ksim_disk_name(int disk);
int ksim_disk_remove(int disk, int replace);
void ksim_disk_stats(int disk, uint64_t *ios, uint64_t *sectors, int64_t *inflight);

int ksim_fs_new(int disk, uint64_t part_start_sect, const char *fstype, int blkbits);
int ksim_file_new(int fs, uint64_t size, const uint8_t *content, const uint64_t *blkmap,
		  uint64_t nblocks);
int ksim_file_open(int file, int readable);
void ksim_pc_set(int file, uint64_t page, int state);
int ksim_pc_get(int file, uint64_t page);
void ksim_file_write(int file, uint64_t off, const uint8_t *src, uint64_t len);
const uint8_t *ksim_file_data(int file);

int ksim_dmabuf_new(uint64_t size, int nsegs, unsigned int seed);
uint8_t *ksim_dmabuf_mem(int fd);
void ksim_dmabuf_state(int fd, int *pinned, int *attached, int *mapped, int *refs);
void ksim_dmabuf_deny_p2p(int fd, int deny);

int ksim_dev_open(int via_proc);
long ksim_ioctl(int fd, unsigned int cmd, void *arg);
long ksim_read(int fd, void *buf, uint64_t n);
int ksim_close(int fd);
const char *ksim_fd_name(int fd);
unsigned long ksim_mmap(int fd, uint64_t len, uint64_t off, int shared);
int ksim_last_mmap_rc(void);   /* the mmap handler's error of the last failed ksim_mmap */
int ksim_munmap(unsigned long addr);
int ksim_user_read(unsigned long addr, void *dst, uint64_t len);
#endif
