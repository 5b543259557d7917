#!/bin/bash
TAG=r04_s12 STAGES="tests smoke bench prof proft" bash tools/evidence.sh
