// Links the in-tree libsplinter.so built by `make host` (or `make all`).
//
// The reference crates compile a vendored copy of splinter.c with `cc` and run
// bindgen over splinter.h (/root/reference/bindings/rust/libsplinter-sys/build.rs:12-37).
// Here the library is a C++ build with an HBM backend that needs the HIP
// runtime, so the crate links the built shared library instead of vendoring
// sources, and the declarations in src/lib.rs are written by hand against the
// frozen ABI (tests/test_bindings_cpu.py checks them against splinter.h).
//
// SPLINTER_LIB_DIR overrides the search path (default: ../../../libsplinter_amd/lib).
use std::env;
use std::path::PathBuf;

fn main() {
    let dir = env::var("SPLINTER_LIB_DIR").map(PathBuf::from).unwrap_or_else(|_| {
        let here = PathBuf::from(env::var("CARGO_MANIFEST_DIR").unwrap());
        here.join("../../../libsplinter_amd/lib")
    });
    println!("cargo:rerun-if-env-changed=SPLINTER_LIB_DIR");
    println!("cargo:rustc-link-search=native={}", dir.display());
    let lib = if env::var("CARGO_FEATURE_PERSISTENT").is_ok() { "splinter_p" } else { "splinter" };
    println!("cargo:rustc-link-lib=dylib={}", lib);
    println!("cargo:rustc-link-arg=-Wl,-rpath,{}", dir.display());
}
