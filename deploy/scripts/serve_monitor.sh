#!/bin/bash
exec python -m finetune_controller_amd.controlplane.monitor "$@"
