/**
 * TypeScript FFI binding for libsplinter_amd (Deno and Bun).
 *
 * Same surface as the reference binding's SplinterStore
 * (/root/reference/bindings/ts/splinter.ts:50-68): open/close/set/get/getString/
 * unset/getEpoch/setLabel/setNamedType/getSignalCount/watchRegister/
 * watchLabelRegister/bumpSlot/getEmbedding/setEmbedding/append/list, over the
 * byte-identical C ABI in libsplinter.so.  Differences: `get` sizes its buffer
 * from the store header (no fixed 4096-B cap), `list` copies key strings out of
 * the library instead of walking raw pointers, the library path comes from
 * SPLINTER_LIB (default ./libsplinter_amd/lib/libsplinter.so), and `hbm:NAME`
 * stores work through the same calls.  Not exercised in this repository's CI
 * (no Deno/Bun in the build image).
 */

export const EMBED_DIM = 768;

const SYMBOLS = {
  splinter_open: { parameters: ["buffer"], result: "i32" },
  splinter_close: { parameters: [], result: "void" },
  splinter_set: { parameters: ["buffer", "buffer", "usize"], result: "i32" },
  splinter_get: { parameters: ["buffer", "buffer", "usize", "buffer"], result: "i32" },
  splinter_unset: { parameters: ["buffer"], result: "i32" },
  splinter_get_epoch: { parameters: ["buffer"], result: "u64" },
  splinter_set_label: { parameters: ["buffer", "u64"], result: "i32" },
  splinter_set_named_type: { parameters: ["buffer", "u16"], result: "i32" },
  splinter_get_signal_count: { parameters: ["u8"], result: "u64" },
  splinter_watch_register: { parameters: ["buffer", "u8"], result: "i32" },
  splinter_watch_label_register: { parameters: ["u64", "u8"], result: "i32" },
  splinter_bump_slot: { parameters: ["buffer"], result: "i32" },
  splinter_get_embedding: { parameters: ["buffer", "buffer"], result: "i32" },
  splinter_set_embedding: { parameters: ["buffer", "buffer"], result: "i32" },
  splinter_append: { parameters: ["buffer", "buffer", "usize", "buffer"], result: "i32" },
  splinter_get_header_snapshot: { parameters: ["buffer"], result: "i32" },
  spl_list_copy: { parameters: ["buffer", "usize"], result: "i64" },
  // host-array batches (splinter_ext.h spl_*_batch) on the current store
  spl_store_current: { parameters: [], result: "pointer" },
  spl_set_batch: {
    parameters: ["pointer", "buffer", "i32", "buffer", "i32", "buffer", "i64", "buffer", "i32", "i32"],
    result: "i64",
  },
  spl_get_batch: {
    parameters: ["pointer", "buffer", "i32", "buffer", "i32", "buffer", "i64", "buffer", "i32", "i32"],
    result: "i64",
  },
} as const;

type Lib = Record<keyof typeof SYMBOLS, (...a: unknown[]) => any>;

const enc = new TextEncoder();
const dec = new TextDecoder();
const cstr = (s: string) => enc.encode(s + "\0");

function loadLib(path: string): Lib {
  // deno-lint-ignore no-explicit-any
  const g = globalThis as any;
  if (g.Deno?.dlopen) return g.Deno.dlopen(path, SYMBOLS).symbols as Lib;
  if (g.Bun) {
    // bun:ffi uses the same type names for these signatures ("buffer" -> "ptr")
    // deno-lint-ignore no-explicit-any
    const { dlopen, FFIType } = require("bun:ffi") as any;
    const map = (t: string) =>
      t === "buffer" || t === "pointer" ? FFIType.ptr : t === "usize" ? FFIType.u64 : (FFIType as any)[t];
    const defs: Record<string, unknown> = {};
    for (const [k, v] of Object.entries(SYMBOLS)) {
      defs[k] = { args: v.parameters.map(map), returns: map(v.result) };
    }
    return dlopen(path, defs).symbols as Lib;
  }
  throw new Error("splinter.ts needs Deno or Bun");
}

export class SplinterStore {
  private lib: Lib;
  private maxVal = 4096;

  private constructor(lib: Lib) {
    this.lib = lib;
  }

  static connect(name: string, libPath?: string): SplinterStore {
    // deno-lint-ignore no-explicit-any
    const env = (globalThis as any).Deno?.env?.get?.("SPLINTER_LIB") ?? (globalThis as any).process?.env?.SPLINTER_LIB;
    const s = new SplinterStore(loadLib(libPath ?? env ?? "./libsplinter_amd/lib/libsplinter.so"));
    s.open(name);
    return s;
  }

  open(name: string): void {
    if (this.lib.splinter_open(cstr(name)) !== 0) throw new Error(`splinter_open(${name}) failed`);
    const hdr = new Uint8Array(48);  // splinter_header_snapshot_t: magic, version, slots, max_val_sz, ...
    if (this.lib.splinter_get_header_snapshot(hdr) === 0) {
      this.maxVal = new DataView(hdr.buffer).getUint32(12, true) || 4096;
    }
  }

  close(): void {
    this.lib.splinter_close();
  }

  set(key: string, value: string | Uint8Array): boolean {
    const v = typeof value === "string" ? enc.encode(value) : value;
    return this.lib.splinter_set(cstr(key), v, BigInt(v.length)) === 0;
  }

  get(key: string): Uint8Array | null {
    const buf = new Uint8Array(this.maxVal);
    const n = new BigUint64Array(1);
    if (this.lib.splinter_get(cstr(key), buf, BigInt(buf.length), new Uint8Array(n.buffer)) !== 0) return null;
    return buf.slice(0, Number(n[0]));
  }

  getString(key: string): string | null {
    const v = this.get(key);
    return v === null ? null : dec.decode(v);
  }

  unset(key: string): number {
    return this.lib.splinter_unset(cstr(key));
  }

  getEpoch(key: string): bigint {
    return BigInt(this.lib.splinter_get_epoch(cstr(key)));
  }

  setLabel(key: string, mask: bigint): boolean {
    return this.lib.splinter_set_label(cstr(key), mask) === 0;
  }

  setNamedType(key: string, mask: number): boolean {
    return this.lib.splinter_set_named_type(cstr(key), mask) === 0;
  }

  getSignalCount(group: number): bigint {
    return BigInt(this.lib.splinter_get_signal_count(group));
  }

  watchRegister(key: string, group: number): boolean {
    return this.lib.splinter_watch_register(cstr(key), group) === 0;
  }

  watchLabelRegister(mask: bigint, group: number): boolean {
    return this.lib.splinter_watch_label_register(mask, group) === 0;
  }

  bumpSlot(key: string): boolean {
    return this.lib.splinter_bump_slot(cstr(key)) === 0;
  }

  getEmbedding(key: string): Float32Array | null {
    const v = new Float32Array(EMBED_DIM);
    return this.lib.splinter_get_embedding(cstr(key), new Uint8Array(v.buffer)) === 0 ? v : null;
  }

  setEmbedding(key: string, vec: Float32Array): boolean {
    if (vec.length !== EMBED_DIM) throw new Error(`embedding must have ${EMBED_DIM} floats`);
    return this.lib.splinter_set_embedding(cstr(key), new Uint8Array(vec.buffer, vec.byteOffset, vec.byteLength)) === 0;
  }

  append(key: string, data: string | Uint8Array): bigint | null {
    const d = typeof data === "string" ? enc.encode(data) : data;
    const n = new BigUint64Array(1);
    if (this.lib.splinter_append(cstr(key), d, BigInt(d.length), new Uint8Array(n.buffer)) !== 0) return null;
    return n[0];
  }

  /** All keys; spl_list_copy writes NUL-separated key names into the buffer. */
  list(): string[] {
    let cap = 1 << 16;
    for (;;) {
      const buf = new Uint8Array(cap);
      const n = Number(this.lib.spl_list_copy(buf, BigInt(cap)));
      if (n < 0) {
        cap = -n;
        continue;
      }
      return dec.decode(buf.subarray(0, n)).split("\0").filter((k) => k.length > 0);
    }
  }
}

/** Fixed-stride records for the batch calls: NUL-padded keys of `kstride` bytes, values of `vstride`. */
function records(items: (string | Uint8Array)[], stride: number): Uint8Array {
  const out = new Uint8Array(items.length * stride);
  items.forEach((it, i) => {
    const b = typeof it === "string" ? enc.encode(it) : it;
    out.set(b.subarray(0, Math.min(b.length, stride)), i * stride);
  });
  return out;
}

/** Batched set / get through the host-array ABI (hbm: / node: stores run them on the GPUs). */
export function setBatch(store: SplinterStore, keys: string[], values: (string | Uint8Array)[], threads = 8): Int32Array {
  // deno-lint-ignore no-explicit-any
  const lib = (store as any).lib as Lib;
  const vb = values.map((v) => (typeof v === "string" ? enc.encode(v) : v));
  const vstride = Math.max(16, Math.ceil(Math.max(1, ...vb.map((v) => v.length)) / 16) * 16);
  const lens = new Uint32Array(vb.map((v) => v.length));
  const status = new Int32Array(keys.length);
  lib.spl_set_batch(lib.spl_store_current(), records(keys.map((k) => k + "\0"), 64), 64, records(vb, vstride),
    vstride, new Uint8Array(lens.buffer), BigInt(keys.length), new Uint8Array(status.buffer), 64, threads);
  return status;
}

export function getBatch(store: SplinterStore, keys: string[], width = 4096, threads = 8):
  { status: Int32Array; values: (Uint8Array | null)[] } {
  // deno-lint-ignore no-explicit-any
  const lib = (store as any).lib as Lib;
  const out = new Uint8Array(keys.length * width);
  const lens = new Uint32Array(keys.length);
  const status = new Int32Array(keys.length);
  lib.spl_get_batch(lib.spl_store_current(), records(keys.map((k) => k + "\0"), 64), 64, out, width,
    new Uint8Array(lens.buffer), BigInt(keys.length), new Uint8Array(status.buffer), 64, threads);
  const values = Array.from(keys, (_, i) => (status[i] === 0 ? out.slice(i * width, i * width + lens[i]) : null));
  return { status, values };
}

/** Polls a signal group (the reference binding's SplinterWatcher.nextSignal, 50 ms cadence). */
export class SplinterWatcher {
  constructor(private store: SplinterStore, private group: number, private pollMs = 50) {}

  async nextSignal(timeoutMs = 0): Promise<bigint | null> {
    const start = this.store.getSignalCount(this.group);
    const t0 = Date.now();
    for (;;) {
      const c = this.store.getSignalCount(this.group);
      if (c !== start) return c;
      if (timeoutMs > 0 && Date.now() - t0 >= timeoutMs) return null;
      await new Promise((r) => setTimeout(r, this.pollMs));
    }
  }
}
