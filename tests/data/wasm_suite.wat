;; miniwasm conformance module for tests/test_cli.py::test_wasm_suite.
;; Each check stores its result (little-endian) under a key via splinter.set.
(module
  (import "splinter" "set" (func $set (param i32 i32 i32 i32) (result i32)))
  (import "splinter" "get" (func $get (param i32 i32 i32) (result i32)))
  (type $bin (func (param i32 i32) (result i32)))
  (memory (export "memory") 1)
  (global $counter (mut i32) (i32.const 0))
  (table 2 funcref)
  (elem (i32.const 0) $add $mul)
  (data (i32.const 0) "fact")      ;; 0..3
  (data (i32.const 8) "fib")       ;; 8..10
  (data (i32.const 16) "tbl")      ;; 16..18
  (data (i32.const 24) "i64")      ;; 24..26
  (data (i32.const 32) "flt")      ;; 32..34
  (data (i32.const 40) "ind")      ;; 40..42
  (data (i32.const 48) "cnt")      ;; 48..50
  (data (i32.const 56) "echo")     ;; 56..59
  (data (i32.const 64) "src")      ;; 64..66

  (func $add (type $bin) (i32.add (local.get 0) (local.get 1)))
  (func $mul (type $bin) (i32.mul (local.get 0) (local.get 1)))

  (func $fact (param $n i64) (result i64)
    (if (result i64) (i64.le_u (local.get $n) (i64.const 1))
      (then (i64.const 1))
      (else (i64.mul (local.get $n) (call $fact (i64.sub (local.get $n) (i64.const 1)))))))

  (func $fib (param $n i32) (result i32)
    (local $a i32) (local $b i32) (local $t i32)
    i32.const 1
    local.set $b
    block $done
      loop $next
        local.get $n
        i32.eqz
        br_if $done
        local.get $a
        local.get $b
        i32.add
        local.set $t
        local.get $b
        local.set $a
        local.get $t
        local.set $b
        local.get $n
        i32.const 1
        i32.sub
        local.set $n
        br $next
      end
    end
    local.get $a)

  (func $classify (param i32) (result i32)
    (block $c (block $b (block $a
      (br_table $a $b $c (local.get 0)))
      (return (i32.const 100)))
      (return (i32.const 200)))
    (i32.const 300))

  (func $put32 (param $key i32) (param $klen i32) (param $v i32)
    (i32.store (i32.const 1024) (local.get $v))
    (drop (call $set (local.get $key) (local.get $klen) (i32.const 1024) (i32.const 4))))

  (func (export "run") (result i32)
    ;; fact(20) as i64
    (i64.store (i32.const 1024) (call $fact (i64.const 20)))
    (drop (call $set (i32.const 0) (i32.const 4) (i32.const 1024) (i32.const 8)))
    (call $put32 (i32.const 8) (i32.const 3) (call $fib (i32.const 30)))
    ;; br_table: 0 -> 100, 1 -> 200, 7 (default) -> 300; packed as 100 + 200*1000 + 300*1000000
    (call $put32 (i32.const 16) (i32.const 3)
      (i32.add (call $classify (i32.const 0))
        (i32.add (i32.mul (call $classify (i32.const 1)) (i32.const 1000))
                 (i32.mul (call $classify (i32.const 7)) (i32.const 1000000)))))
    ;; i64 shifts / rotates / div: (-9 >> 1) signed, rotl, unsigned div
    (i64.store (i32.const 1024) (i64.add (i64.shr_s (i64.const -9) (i64.const 1))
                                         (i64.add (i64.rotl (i64.const 1) (i64.const 63))
                                                  (i64.div_u (i64.const -1) (i64.const 3)))))
    (drop (call $set (i32.const 24) (i32.const 3) (i32.const 1024) (i32.const 8)))
    ;; floats: trunc(sqrt(2) * 1e6) and f32 min/max/nearest
    (call $put32 (i32.const 32) (i32.const 3)
      (i32.add (i32.trunc_f64_s (f64.mul (f64.sqrt (f64.const 2)) (f64.const 1e6)))
               (i32.trunc_f32_s (f32.nearest (f32.max (f32.const 2.5) (f32.min (f32.const -1) (f32.const 3.5)))))))
    ;; call_indirect through the table: add(6,7) * mul(6,7)
    (call $put32 (i32.const 40) (i32.const 3)
      (i32.mul (call_indirect (type $bin) (i32.const 6) (i32.const 7) (i32.const 0))
               (call_indirect (type $bin) (i32.const 6) (i32.const 7) (i32.const 1))))
    ;; globals + memory.grow / memory.size + sign extension
    (global.set $counter (i32.add (global.get $counter) (i32.const 5)))
    (drop (memory.grow (i32.const 2)))
    (call $put32 (i32.const 48) (i32.const 3)
      (i32.add (i32.mul (global.get $counter) (i32.const 100))
               (i32.add (memory.size) (i32.extend8_s (i32.const 0xff)))))
    ;; host get: copy key "src" to "echo"
    (call $set (i32.const 56) (i32.const 4) (i32.const 2048) (call $get (i32.const 64) (i32.const 3) (i32.const 2048))))

  (func (export "trap") (result i32)
    (i32.div_s (i32.const 1) (i32.const 0)))
)
