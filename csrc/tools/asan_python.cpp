// Python interpreter entry point linked with the ASan/UBSan runtimes (csrc/build.py
// build_asan_python): running the test suite through it puts the sanitizer runtime first
// in the process, so the instrumented host binding layer (_C_san.so) can be imported
// without touching the dynamic loader's preload list.
#include <Python.h>

int main(int argc, char** argv) { return Py_BytesMain(argc, argv); }
