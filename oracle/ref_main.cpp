// TEST INFRASTRUCTURE ONLY: entry point of oracle/_ref/ref_dump (the harness
// TU renames the reference app's own main to reference_main).
int harness_main(int argc, char** argv);
int main(int argc, char** argv) { return harness_main(argc, argv); }
