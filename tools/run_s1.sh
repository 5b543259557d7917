#!/bin/bash
TAG=r04_s35 STAGES="tests smoke bench prof proft" bash tools/evidence.sh
