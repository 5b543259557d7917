#!/bin/bash
TAG=r04_s22 STAGES="tests smoke bench prof proft" bash tools/evidence.sh
