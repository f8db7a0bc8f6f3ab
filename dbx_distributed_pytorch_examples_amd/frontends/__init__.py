"""Reference-compatible API adapters over the one engine (SURVEY.md §1 L6 launchers):
TorchDistributor / DeepSpeed / Composer / Accelerate / Ray Train styles."""
