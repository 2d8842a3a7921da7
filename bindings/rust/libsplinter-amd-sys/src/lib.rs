//! Raw FFI bindings to libsplinter_amd: the splinter.h C ABI (format v4).
//!
//! Declarations mirror `libsplinter_amd/csrc/include/splinter.h` one to one
//! (the reference crate binds the same 60 calls through bindgen,
//! /root/reference/bindings/rust/libsplinter-sys/src/lib.rs:11).  Store names
//! select the backend at run time: `"name"` = POSIX shm, a path or `file:` =
//! regular file, `"hbm:name"` = the arena in the HBM of an MI355X.
//!
//! Layout structs are `#[repr(C)]` with the same alignment as the header; the
//! byte offsets are pinned by `splinter_layout.hpp` static_asserts on the C++
//! side and by the `layout` test below.
#![allow(non_camel_case_types)]

use std::os::raw::{c_char, c_int, c_long, c_uint, c_ushort, c_void};

pub const SPLINTER_MAGIC: u32 = 0x534C_4E54;
pub const SPLINTER_VER: u32 = 4;
pub const SPLINTER_KEY_MAX: usize = 64;
pub const SPLINTER_EMBED_DIM: usize = 768;
pub const SPLINTER_MAX_GROUPS: usize = 64;
pub const SPLINTER_MAX_SHARDS: usize = 32;
pub const SPLINTER_MAX_SLOTS: usize = 1024;
pub const SPLINTER_EVENT_BUS_MASK_WORDS: usize = SPLINTER_MAX_SLOTS / 64;

pub const SPL_SYS_AUTO_SCRUB: u8 = 1 << 0;
pub const SPL_SYS_HYBRID_SCRUB: u8 = 1 << 1;

pub const SPL_SLOT_TYPE_VOID: u16 = 1 << 0;
pub const SPL_SLOT_TYPE_BIGINT: u16 = 1 << 1;
pub const SPL_SLOT_TYPE_BIGUINT: u16 = 1 << 2;
pub const SPL_SLOT_TYPE_JSON: u16 = 1 << 3;
pub const SPL_SLOT_TYPE_BINARY: u16 = 1 << 4;
pub const SPL_SLOT_TYPE_IMGDATA: u16 = 1 << 5;
pub const SPL_SLOT_TYPE_AUDIO: u16 = 1 << 6;
pub const SPL_SLOT_TYPE_VARTEXT: u16 = 1 << 7;

pub const SPL_TIME_CTIME: c_ushort = 0;
pub const SPL_TIME_ATIME: c_ushort = 1;

pub type splinter_intent_t = c_uint;
pub const SPL_INTENT_NONE: splinter_intent_t = 0;
pub const SPL_INTENT_WILLNEED: splinter_intent_t = 1;
pub const SPL_INTENT_SEQUENTIAL: splinter_intent_t = 2;
pub const SPL_INTENT_RANDOM: splinter_intent_t = 3;
pub const SPL_INTENT_DONTNEED: splinter_intent_t = 4;

pub type splinter_integer_op_t = c_uint;
pub const SPL_OP_AND: splinter_integer_op_t = 0;
pub const SPL_OP_OR: splinter_integer_op_t = 1;
pub const SPL_OP_XOR: splinter_integer_op_t = 2;
pub const SPL_OP_NOT: splinter_integer_op_t = 3;
pub const SPL_OP_INC: splinter_integer_op_t = 4;
pub const SPL_OP_DEC: splinter_integer_op_t = 5;

#[repr(C, align(64))]
#[derive(Debug, Copy, Clone)]
pub struct splinter_signal_node {
    pub counter: u64,
}

#[repr(C)]
#[derive(Debug, Copy, Clone)]
pub struct splinter_event_bus {
    pub dirty_mask: [u64; SPLINTER_EVENT_BUS_MASK_WORDS],
    pub owner_fd: i32,
    pub owner_pid: i32,
}

#[repr(C)]
#[derive(Debug, Copy, Clone)]
pub struct splinter_shard_bid {
    pub shard_id: u32,
    pub pid: u32,
    pub intent: u8,
    pub priority: u8,
    pub _pad: [u8; 2],
    pub duration_tsc: u64,
    pub claimed_at: u64,
}

#[repr(C, align(64))]
#[derive(Debug, Copy, Clone)]
pub struct Aligned64<T: Copy>(pub T);

#[repr(C)]
pub struct splinter_header {
    pub magic: u32,
    pub version: u32,
    pub slots: u32,
    pub max_val_sz: u32,
    pub epoch: u64,
    pub core_flags: u8,
    pub user_flags: u8,
    pub val_brk: u32,
    pub val_sz: u32,
    pub alignment: u32,
    pub parse_failures: u64,
    pub last_failure_epoch: u64,
    pub bloom_watches: [u8; 64],
    pub signal_groups: [splinter_signal_node; SPLINTER_MAX_GROUPS],
    pub event_bus: Aligned64<splinter_event_bus>,
    pub shard_bids: Aligned64<[splinter_shard_bid; SPLINTER_MAX_SHARDS]>,
}

#[repr(C, align(64))]
pub struct splinter_slot {
    pub hash: u64,
    pub epoch: u64,
    pub val_off: u32,
    pub val_len: u32,
    pub type_flag: u8,
    pub user_flag: u8,
    pub watcher_mask: u64,
    pub ctime: u64,
    pub atime: u64,
    pub bloom: u64,
    pub key: [c_char; SPLINTER_KEY_MAX],
}

#[repr(C)]
#[derive(Debug, Copy, Clone, Default)]
pub struct splinter_header_snapshot_t {
    pub magic: u32,
    pub version: u32,
    pub slots: u32,
    pub max_val_sz: u32,
    pub epoch: u64,
    pub core_flags: u8,
    pub user_flags: u8,
    pub parse_failures: u64,
    pub last_failure_epoch: u64,
}

#[repr(C)]
#[derive(Copy, Clone)]
pub struct splinter_slot_snapshot_t {
    pub hash: u64,
    pub epoch: u64,
    pub val_off: u32,
    pub val_len: u32,
    pub type_flag: u8,
    pub user_flag: u8,
    pub ctime: u64,
    pub atime: u64,
    pub bloom: u64,
    pub key: [c_char; SPLINTER_KEY_MAX],
    pub embedding: [f32; SPLINTER_EMBED_DIM],
}

#[repr(C)]
#[derive(Debug, Copy, Clone, Default)]
pub struct splinter_shard_bid_snapshot {
    pub shard_id: u32,
    pub pid: u32,
    pub intent: u8,
    pub priority: u8,
    pub duration_tsc: u64,
    pub claimed_at: u64,
    pub expired: c_int,
    pub sovereign: c_int,
}

pub type splinter_enum_cb = Option<unsafe extern "C" fn(key: *const c_char, epoch: u64, data: *mut c_void)>;

extern "C" {
    // lifecycle
    pub fn splinter_create(name_or_path: *const c_char, slots: usize, max_value_sz: usize) -> c_int;
    pub fn splinter_open(name_or_path: *const c_char) -> c_int;
    pub fn splinter_open_numa(name: *const c_char, target_node: c_int) -> *mut c_void;
    pub fn splinter_open_or_create(name_or_path: *const c_char, slots: usize, max_value_sz: usize) -> c_int;
    pub fn splinter_create_or_open(name_or_path: *const c_char, slots: usize, max_value_sz: usize) -> c_int;
    pub fn splinter_close();
    // store-wide
    pub fn splinter_set_mop(mode: c_uint) -> c_int;
    pub fn splinter_get_mop() -> c_int;
    pub fn splinter_purge();
    pub fn splinter_get_header_snapshot(snapshot: *mut splinter_header_snapshot_t) -> c_int;
    // key/value
    pub fn splinter_set(key: *const c_char, val: *const c_void, len: usize) -> c_int;
    pub fn splinter_unset(key: *const c_char) -> c_int;
    pub fn splinter_get(key: *const c_char, buf: *mut c_void, buf_sz: usize, out_sz: *mut usize) -> c_int;
    pub fn splinter_list(out_keys: *mut *mut c_char, max_keys: usize, out_count: *mut usize) -> c_int;
    pub fn splinter_poll(key: *const c_char, timeout_ms: u64) -> c_int;
    pub fn splinter_get_slot_snapshot(key: *const c_char, snapshot: *mut splinter_slot_snapshot_t) -> c_int;
    pub fn splinter_append(key: *const c_char, data: *const c_void, data_len: usize, new_len: *mut usize) -> c_int;
    pub fn splinter_get_raw_ptr(key: *const c_char, out_sz: *mut usize, out_epoch: *mut u64) -> *const c_void;
    pub fn splinter_get_epoch(key: *const c_char) -> u64;
    pub fn splinter_set_as_system(key: *const c_char) -> c_int;
    // embeddings
    pub fn splinter_set_embedding(key: *const c_char, embedding: *const f32) -> c_int;
    pub fn splinter_get_embedding(key: *const c_char, embedding_out: *mut f32) -> c_int;
    // flags
    pub fn splinter_config_set(hdr: *mut splinter_header, mask: u8);
    pub fn splinter_config_clear(hdr: *mut splinter_header, mask: u8);
    pub fn splinter_config_test(hdr: *mut splinter_header, mask: u8) -> c_int;
    pub fn splinter_config_snapshot(hdr: *mut splinter_header) -> u8;
    pub fn splinter_slot_usr_set(slot: *mut splinter_slot, mask: u16);
    pub fn splinter_slot_usr_clear(slot: *mut splinter_slot, mask: u16);
    pub fn splinter_slot_usr_test(slot: *mut splinter_slot, mask: u16) -> c_int;
    pub fn splinter_slot_usr_snapshot(slot: *mut splinter_slot) -> u16;
    // typing, time, integers
    pub fn splinter_set_named_type(key: *const c_char, mask: u16) -> c_int;
    pub fn splinter_set_slot_time(key: *const c_char, mode: c_ushort, epoch: u64, offset: usize) -> c_int;
    pub fn splinter_integer_op(key: *const c_char, op: splinter_integer_op_t, mask: *const c_void) -> c_int;
    pub fn splinter_now_ticks() -> u64;
    // epochs, labels, tandem
    pub fn splinter_bump_slot(key: *const c_char) -> c_int;
    pub fn splinter_retrain_slot(key: *const c_char) -> c_int;
    pub fn splinter_set_label(key: *const c_char, mask: u64) -> c_int;
    pub fn splinter_unset_label(key: *const c_char, mask: u64) -> c_int;
    pub fn splinter_client_set_tandem(base_key: *const c_char, vals: *mut *const c_void, lens: *const usize,
                                      orders: u8) -> c_int;
    pub fn splinter_client_unset_tandem(base_key: *const c_char, orders: u8);
    // signals
    pub fn splinter_watch_register(key: *const c_char, group_id: u8) -> c_int;
    pub fn splinter_watch_unregister(key: *const c_char, group_id: u8) -> c_int;
    pub fn splinter_watch_label_register(bloom_mask: u64, group_id: u8) -> c_int;
    pub fn splinter_pulse_watchers(slot: *mut splinter_slot);
    pub fn splinter_pulse_keygroup(key: *const c_char) -> c_int;
    pub fn splinter_get_signal_count(group_id: u8) -> u64;
    pub fn splinter_enumerate_matches(mask: u64, callback: splinter_enum_cb, user_data: *mut c_void);
    // event bus
    pub fn splinter_event_bus_init() -> c_int;
    pub fn splinter_event_bus_open() -> c_int;
    pub fn splinter_event_bus_wait(fd: c_int, timeout_ms: u64) -> c_int;
    pub fn splinter_event_bus_close(fd: c_int);
    pub fn splinter_event_bus_get_dirty(out: *mut u64, words: usize);
    // logic shard election / cooperative madvise
    pub fn splinter_shard_claim(shard_id: u32, intent: u8, priority: u8, duration_tsc: u64) -> c_int;
    pub fn splinter_shard_claim_ex(shard_id: u32, pid: u32, intent: u8, priority: u8, duration_tsc: u64,
                                   claimed_at: u64) -> c_int;
    pub fn splinter_shard_rebid(shard_id: u32, intent: u8, priority: u8, duration_tsc: u64) -> c_int;
    pub fn splinter_shard_release(shard_id: u32) -> c_int;
    pub fn splinter_shard_election(out_intent: *mut u8) -> u32;
    pub fn splinter_shard_is_sovereign(shard_id: u32) -> c_int;
    pub fn splinter_shard_table_snapshot(out: *mut splinter_shard_bid_snapshot, max: usize) -> c_int;
    pub fn splinter_madvise(shard_id: u32, addr: *mut c_void, len: usize, advice: c_int, timeout_ticks: u64) -> c_int;
}

/// `splinter_now` is a static inline in splinter.h; this is its FFI-visible twin.
#[inline]
pub unsafe fn splinter_now() -> u64 {
    splinter_now_ticks()
}

#[cfg(test)]
mod layout {
    use super::*;
    use std::mem::{align_of, size_of};

    #[test]
    fn format_v4_sizes() {
        // the same numbers splinter_layout.hpp pins with static_asserts
        assert_eq!(size_of::<splinter_slot>(), 128);
        assert_eq!(align_of::<splinter_slot>(), 64);
        assert_eq!(size_of::<splinter_header>(), 5440);
        assert_eq!(size_of::<splinter_header_snapshot_t>(), 48);
        assert_eq!(size_of::<splinter_shard_bid_snapshot>(), 40);
    }
}

/// Opaque handle of the libsplinter_amd extension API (splinter_ext.h).
#[repr(C)]
pub struct spl_store {
    _private: [u8; 0],
}

// Host-array batches (splinter_ext.h spl_*_batch): fixed-stride NUL-padded key records, value rows
// of vstride / ostride bytes, per-op status 0 / -errno; hbm: / node: stores run them on the GPUs.
extern "C" {
    pub fn spl_store_current() -> *mut spl_store;
    pub fn spl_set_batch(s: *mut spl_store, keys: *const c_char, kstride: c_int, vals: *const u8, vstride: c_int,
                         lens: *const u32, n: c_long, status: *mut i32, retries: c_int, threads: c_int) -> c_long;
    pub fn spl_get_batch(s: *mut spl_store, keys: *const c_char, kstride: c_int, out: *mut u8, ostride: c_int,
                         out_lens: *mut u32, n: c_long, status: *mut i32, retries: c_int, threads: c_int) -> c_long;
    pub fn spl_intop_batch_ex(s: *mut spl_store, keys: *const c_char, kstride: c_int, ops: *const c_int,
                              masks: *const u64, n: c_long, status: *mut i32, results: *mut u64, threads: c_int)
                              -> c_long;
    pub fn spl_set_embedding_batch(s: *mut spl_store, keys: *const c_char, kstride: c_int, vecs: *const f32,
                                   n: c_long, expect_epochs: *const u64, status: *mut i32, threads: c_int) -> c_long;
    pub fn spl_batch_alloc(bytes: usize) -> *mut c_void;
    pub fn spl_batch_free(p: *mut c_void);
}

// libsplinter_hip.so (loaded by libsplinter.so on the first hbm: / node: store): the per-call ring
extern "C" {
    pub fn spl_hbm_ring_mode(s: *mut spl_store) -> c_int;
    pub fn spl_ring_hold(on: c_int);
    pub fn spl_hbm_ring_hold(s: *mut spl_store, on: c_int) -> c_int;
}
