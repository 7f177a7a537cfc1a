"""`pkbench.gb` — the synthetic game ROM the benchmark runs (pokemon_red.gb is not shipped).

It is a small overworld RPG built to exercise the emulator the way Pokémon Red's frame loop does
(pokered's main loop structure: DelayFrame HALT wait, VBlank handler with OAM DMA from an HRAM
routine, AutoBgMapTransfer of a third of the WRAM tile map per frame, a table-driven sound
engine in a switched ROM bank, ReadJoypad, the DIV-mixing Random routine; then overworld logic):
  * player movement on a 64x64 metatile map with collision (held d-pad = one step per 8 frames),
    full 20x18 map-view redraw into the WRAM tile map after every step,
  * 8 NPCs doing RNG random walks with collision, 36 sprites rebuilt into the OAM buffer,
  * a text engine (A opens a box, one character per frame, A closes it; B speeds it up),
  * random encounters on grass that run a battle engine in ROM bank 3 (16-bit Multiply and
    bit-serial Divide like pokered's home/math routines, damage formula, HP bars into the tile
    map) and decompress a 392-byte "sprite" into cartridge SRAM (pokered's sSpriteBuffer),
  * START toggles a menu that re-draws part of the screen, SELECT swaps palettes.
Everything is deterministic given the action stream; per-env divergence comes from the actions
(RNG mixes DIV, which is identical across envs at equal cycle counts).
"""
from __future__ import annotations

import re

from .sm83asm import build_rom

SRC = r"""
; ---------------------------------------------------------------- constants
rLCDC equ $40
hDMA equ $80
hJoyHeld equ $b4
hJoyPressed equ $b3
hJoyLast equ $b1
hROMBank equ $b8
hVBlankOccurred equ $d6
hFrameCounter equ $d5
hRandomAdd equ $d3
hRandomSub equ $d4
hBGPortion equ $b2
hMoveTimer equ $b5
hTextActive equ $b6
hBattle equ $b7
hMenu equ $b9
wOAM equ $c000
wTileMap equ $c100
wMap equ $c300
wPlayerX equ $d400
wPlayerY equ $d401
wPlayerFacing equ $d402
wMoved equ $d403
wNPC equ $d410
wTextPtr equ $d450
wTextCol equ $d452
wTextRow equ $d453
wBattleHP equ $d460
wBattleEnemyHP equ $d462
wBattleTurn equ $d464
wBattleTimer equ $d465
wMathA equ $d470
wMathB equ $d472
wMathR equ $d474
wSound equ $d480
wStepCount equ $d4a0
wMapSeed equ $d4a1
wSprState equ $d4c0

section 0
org $0000
    ret
org $0008
    ret
org $0040
    jp vblank
org $0048
    reti
org $0050
    reti
org $0058
    reti
org $0060
    reti

org $0100
    nop
    jp start

org $0150
start:
    di
    ld sp, $dfff
    ; LCD off while we set up (pokered DisableLCD waits for LY=145)
.wly:
    ldh a, [$44]
    cp 145
    jr nz, .wly
    xor a
    ldh [rLCDC], a
    ; copy the OAM DMA routine to HRAM
    ld hl, dma_routine
    ld de, $ff80
    ld b, 8
.cpd:
    ld a, [hl+]
    ld [de], a
    inc de
    dec b
    jr nz, .cpd
    ; tiles: 64 tiles of generated 2bpp patterns at $8000 and $9000
    ld hl, $8000
    ld de, $0000
.tile:
    ld a, e
    xor d
    rlca
    add a, d
    ld [hl+], a
    ld a, e
    rrca
    or d
    ld [hl+], a
    inc e
    ld a, e
    and $0f
    jr nz, .tile
    inc d
    ld a, h
    cp $88
    jr nz, .tile
    ; map: 64x64 metatiles from an LFSR; 0-3 floor, 4-5 grass, 6-7 wall
    ld hl, wMap
    ld bc, $1000
    ld e, $5a
.map:
    ld a, e
    add a, a
    jr nc, .nox
    xor $1d
.nox:
    ld e, a
    and $07
    ld [hl+], a
    dec bc
    ld a, b
    or c
    jr nz, .map
    ; player / NPCs
    ld a, 32
    ld [wPlayerX], a
    ld [wPlayerY], a
    ld hl, wNPC
    ld b, 8
    ld a, 20
.npc:
    ld [hl+], a
    add a, 3
    ld [hl+], a
    add a, 5
    ld [hl+], a
    ld [hl+], a
    dec b
    jr nz, .npc
    xor a
    ldh [hJoyHeld], a
    ldh [hJoyPressed], a
    ldh [hTextActive], a
    ldh [hBattle], a
    ldh [hMenu], a
    ldh [hBGPortion], a
    ldh [hMoveTimer], a
    ld a, $5a
    ld [wMapSeed], a
    call set_party
    ld a, 1
    ld [wMoved], a
    ldh [hROMBank], a
    ld [$2000], a
    ; sound channels
    ld hl, wSound
    ld b, 32
    ld a, 1
.snd:
    ld [hl+], a
    inc a
    dec b
    jr nz, .snd
    ; palettes, LCD on: BG + window ($9c00) + sprites, tile data at $8000
    ld a, $e4
    ldh [$47], a
    ld a, $d0
    ldh [$48], a
    ld a, $e0
    ldh [$49], a
    ld a, 144
    ldh [$4a], a
    ld a, 7
    ldh [$4b], a
    ld a, $f3
    ldh [rLCDC], a
    ld a, $01
    ldh [$ff], a
    ei

main:
    call delay_frame
    call handle_input
    call update_npcs
    call update_sprites
    ld a, [wMoved]
    and a
    call nz, draw_map_view
    call text_engine
    call menu_logic
    ldh a, [hBattle]
    and a
    jr z, main
    ld a, 3
    call farcall_battle
    jr main

; ---------------------------------------------------------------- home routines
delay_frame:
    ld a, 1
    ldh [hVBlankOccurred], a
.h:
    halt
    ldh a, [hVBlankOccurred]
    and a
    jr nz, .h
    ret

farcall_battle:
    ; pokered Bankswitch: save bank, switch, call, restore
    ld b, a
    ldh a, [hROMBank]
    push af
    ld a, b
    ldh [hROMBank], a
    ld [$2000], a
    call battle_step
    pop af
    ldh [hROMBank], a
    ld [$2000], a
    ret

random:
    ldh a, [$04]
    ld b, a
    ldh a, [hRandomAdd]
    adc a, b
    ldh [hRandomAdd], a
    ldh a, [$04]
    ld b, a
    ldh a, [hRandomSub]
    sbc a, b
    ldh [hRandomSub], a
    ret

; map lookup: d = y, e = x (metatile coords 0..63) -> a = metatile
map_at:
    push hl
    ld a, d
    and $3f
    ld l, a
    ld h, 0
    add hl, hl
    add hl, hl
    add hl, hl
    add hl, hl
    add hl, hl
    add hl, hl
    ld a, e
    and $3f
    add a, l
    ld l, a
    ld a, h
    adc a, $c3
    ld h, a
    ld a, [hl]
    pop hl
    ret

handle_input:
    ldh a, [hTextActive]
    and a
    ret nz
    ldh a, [hBattle]
    and a
    ret nz
    ldh a, [hMoveTimer]
    and a
    jr z, .ready
    dec a
    ldh [hMoveTimer], a
    ret
.ready:
    ldh a, [hJoyHeld]
    and $f0
    ret z
    ld b, a
    ld a, [wPlayerY]
    ld d, a
    ld a, [wPlayerX]
    ld e, a
    bit 4, b
    jr z, .nr
    inc e
    ld c, 1
.nr:
    bit 5, b
    jr z, .nl
    dec e
    ld c, 2
.nl:
    bit 6, b
    jr z, .nu
    dec d
    ld c, 3
.nu:
    bit 7, b
    jr z, .nd
    inc d
    ld c, 0
.nd:
    ld a, c
    ld [wPlayerFacing], a
    call map_at
    cp 6
    ret nc
    ld b, a
    ld a, d
    and $3f
    ld [wPlayerY], a
    ld a, e
    and $3f
    ld [wPlayerX], a
    ld a, 1
    ld [wMoved], a
    ld a, 7
    ldh [hMoveTimer], a
    ld hl, wStepCount
    inc [hl]
    ; a door (floor metatile 3): warp into a new map, loaded with the LCD off
    ld a, b
    cp 3
    jp z, map_warp
    ; grass: random encounter
    ld a, b
    cp 4
    ret c
    call random
    cp 64
    ret nc
    ld a, 1
    ldh [hBattle], a
    ld a, 40
    ld [wBattleHP], a
    ld a, 30
    ld [wBattleEnemyHP], a
    xor a
    ld [wBattleTurn], a
    ret

; pokered's map transition through a door (EnterMap -> LoadMapData): DisableLCD (wait for LY = 145,
; LCD off), the new map's tileset graphics copied into VRAM and its blocks rebuilt in WRAM while the
; LCD is off — several frames of bulk copies with no VBlank, the frames ending on the LCD-off clock
; alone — then EnableLCD and a full map-view redraw
map_warp:
    ld a, [wMapSeed]
    add a, 29
    or 1
    ld [wMapSeed], a
    ; DisableLCD: VBlank interrupt off while waiting for LY = 145 (the handler runs longer than a
    ; scanline, so with it enabled the poll would never see line 145)
    xor a
    ldh [$0f], a
    ldh a, [$ff]
    push af
    res 0, a
    ldh [$ff], a
.wly:
    ldh a, [$44]
    cp 145
    jr nz, .wly
    ldh a, [rLCDC]
    and $7f
    ldh [rLCDC], a
    ; tileset graphics: 2 KiB of bank-0 bytes into tiles 128-255 ($8800-$8fff)
    ld hl, $0100
    ld de, $8800
    ld bc, $0800
.gfx:
    ld a, [hl+]
    ld [de], a
    inc de
    dec bc
    ld a, b
    or c
    jr nz, .gfx
    ; map blocks: the 64x64 metatile map from the new seed (the boot-time LFSR)
    ld hl, wMap
    ld bc, $1000
    ld a, [wMapSeed]
    ld e, a
.blk:
    ld a, e
    add a, a
    jr nc, .nox
    xor $1d
.nox:
    ld e, a
    and $07
    ld [hl+], a
    dec bc
    ld a, b
    or c
    jr nz, .blk
    call set_party
    ldh a, [rLCDC]
    or $80
    ldh [rLCDC], a
    xor a
    ldh [$0f], a
    pop af
    ldh [$ff], a
    ld a, 1
    ld [wMoved], a
    ret

; the party: one level-5 Bulbasaur with 20/20 HP at pokered's wPartyCount/wPartyMons addresses (the
; reference's save states always hold a party — an empty one makes its info step raise,
; environment.py:1672).  They lie inside the 4 KiB map blocks, so every map (re)build rewrites them
set_party:
    ld a, 1
    ld [$d163], a
    ld a, $99
    ld [$d164], a
    ld [$d16b], a
    ld a, $ff
    ld [$d165], a
    ld a, 5
    ld [$d18c], a
    ld a, 20
    ld [$d16d], a
    ld [$d18e], a
    ret

update_npcs:
    ld hl, wNPC
    ld c, 8
.loop:
    call random
    and $0f
    jr nz, .skip
    ldh a, [hRandomSub]
    and 3
    ld b, a
    ld a, [hl+]
    ld d, a
    ld a, [hl-]
    ld e, a
    ld a, b
    cp 0
    jr nz, .a1
    inc e
.a1:
    cp 1
    jr nz, .a2
    dec e
.a2:
    cp 2
    jr nz, .a3
    inc d
.a3:
    cp 3
    jr nz, .a4
    dec d
.a4:
    call map_at
    cp 6
    jr nc, .skip
    ld a, d
    and $3f
    ld [hl+], a
    ld a, e
    and $3f
    ld [hl-], a
.skip:
    inc hl
    inc hl
    inc hl
    inc hl
    dec c
    jr nz, .loop
    ret

; sprite state table wSprState: 9 metasprites x 4 bytes (y, x, tile base, facing),
; positions relative to the player (pokered UpdateSprites -> wSpriteStateData1)
update_sprites:
    ld de, wSprState
    ld a, 72
    ld [de], a
    inc de
    ld a, 80
    ld [de], a
    inc de
    xor a
    ld [de], a
    inc de
    ld a, [wPlayerFacing]
    ld [de], a
    inc de
    ld hl, wNPC
    ld c, 8
.n:
    ld a, [wPlayerY]
    ld b, a
    ld a, [hl+]
    sub b
    add a, a
    add a, a
    add a, a
    add a, a
    add a, 72
    ld [de], a
    inc de
    ld a, [wPlayerX]
    ld b, a
    ld a, [hl+]
    sub b
    add a, a
    add a, a
    add a, a
    add a, a
    add a, 80
    ld [de], a
    inc de
    ld a, $10
    ld [de], a
    inc de
    ld a, [hl+]
    and 3
    ld [de], a
    inc de
    inc hl
    dec c
    jr nz, .n
    ret

; pokered PrepareOAMData: expand the sprite state table into the OAM buffer (9 metasprites x
; 4 tiles) with per-facing tile/flip tables and a walking animation frame
prepare_oam:
    ld hl, wSprState
    ld de, wOAM
    ld a, 9
.spr:
    push af
    ld a, [hl+]
    ld b, a
    ld a, [hl+]
    ld c, a
    inc hl
    ld a, [hl+]
    push hl
    add a, a
    add a, a
    ld hl, oam_attr
    add a, l
    ld l, a
    ld a, h
    adc a, 0
    ld h, a
    call put_tile
    ld a, c
    add a, 8
    ld c, a
    call put_tile
    ld a, b
    add a, 8
    ld b, a
    ld a, c
    sub 8
    ld c, a
    call put_tile
    ld a, c
    add a, 8
    ld c, a
    call put_tile
    pop hl
    pop af
    dec a
    jr nz, .spr
    ret

; one OAM entry at de: y = b, x = c, [hl] = tile (bits 0-4) | flips (bits 5-6); hl += 1
put_tile:
    ld a, b
    add a, 16
    ld [de], a
    inc de
    ld a, c
    add a, 8
    ld [de], a
    inc de
    ldh a, [hFrameCounter]
    and $08
    rrca
    rrca
    rrca
    add a, [hl]
    and $1f
    ld [de], a
    inc de
    ld a, [hl+]
    and $60
    ld [de], a
    inc de
    ret

oam_attr:
    db $00, $02, $04, $06
    db $08, $0a, $0c, $0e
    db $10, $32, $14, $36
    db $38, $1a, $3c, $1e

; rebuild the 20x18 tile map around the player (pokered LoadCurrentMapView)
draw_map_view:
    xor a
    ld [wMoved], a
    ld hl, wTileMap
    ld a, [wPlayerY]
    sub 4
    ld d, a
    ld b, 9
.row:
    ld a, [wPlayerX]
    sub 5
    ld e, a
    ld c, 10
.col:
    call map_at
    add a, a
    add a, a
    ld [hl+], a
    inc a
    ld [hl+], a
    inc e
    dec c
    jr nz, .col
    ; second tile row of the metatiles: copy the row above +2
    push de
    ld d, h
    ld e, l
    ld a, l
    sub 20
    ld l, a
    ld a, h
    sbc a, 0
    ld h, a
    ld c, 20
.cp2:
    ld a, [hl+]
    add a, 2
    ld [de], a
    inc de
    dec c
    jr nz, .cp2
    ld h, d
    ld l, e
    pop de
    inc d
    dec b
    jr nz, .row
    ret

text_engine:
    ldh a, [hTextActive]
    and a
    jr nz, .active
    ldh a, [hJoyPressed]
    bit 0, a
    ret z
    ldh a, [hBattle]
    and a
    ret nz
    ld a, 1
    ldh [hTextActive], a
    ld hl, text_data
    ld a, [wStepCount]
    and $03
    add a, a
    add a, a
    add a, a
    add a, a
    add a, l
    ld l, a
    ld a, h
    adc a, 0
    ld h, a
    ld a, l
    ld [wTextPtr], a
    ld a, h
    ld [wTextPtr + 1], a
    xor a
    ld [wTextCol], a
    ld [wTextRow], a
    ret
.active:
    cp 2
    jr z, .wait_close
    ld a, [wTextPtr]
    ld l, a
    ld a, [wTextPtr + 1]
    ld h, a
    ld a, [hl+]
    and a
    jr z, .done
    ld b, a
    ld a, l
    ld [wTextPtr], a
    ld a, h
    ld [wTextPtr + 1], a
    ; tile map position: row 14 + wTextRow, col 1 + wTextCol
    ld a, [wTextCol]
    inc a
    ld [wTextCol], a
    ld c, a
    ld hl, wTileMap + 20 * 14
    ld a, c
    add a, l
    ld l, a
    ld a, h
    adc a, 0
    ld h, a
    ld [hl], b
    ldh a, [hBGPortion]
    ret
.done:
    ld a, 2
    ldh [hTextActive], a
    ret
.wait_close:
    ldh a, [hJoyPressed]
    and $03
    ret z
    xor a
    ldh [hTextActive], a
    ld a, 1
    ld [wMoved], a
    ret

menu_logic:
    ldh a, [hJoyPressed]
    bit 3, a
    jr z, .sel
    ldh a, [hMenu]
    xor 1
    ldh [hMenu], a
    ; window shows the menu when open
    and a
    ld a, 144
    jr z, .wy
    ld a, 96
.wy:
    ldh [$4a], a
.sel:
    ldh a, [hJoyPressed]
    bit 2, a
    ret z
    ldh a, [$47]
    rlca
    rlca
    ldh [$47], a
    ret

; ---------------------------------------------------------------- VBlank
vblank:
    push af
    push bc
    push de
    push hl
    ldh a, [hROMBank]
    push af
    ld a, $c0
    call $ff80
    call prepare_oam
    call bg_transfer
    ld a, 2
    ldh [hROMBank], a
    ld [$2000], a
    call sound_update
    call read_joypad
    call random
    ldh a, [hFrameCounter]
    inc a
    ldh [hFrameCounter], a
    xor a
    ldh [hVBlankOccurred], a
    pop af
    ldh [hROMBank], a
    ld [$2000], a
    pop hl
    pop de
    pop bc
    pop af
    reti

; pokered AutoBgMapTransfer: one third (6 rows) of the tile map per frame
bg_transfer:
    ldh a, [hBGPortion]
    ld b, a
    inc a
    cp 3
    jr c, .ok
    xor a
.ok:
    ldh [hBGPortion], a
    ld hl, wTileMap
    ld de, $9800
    ld a, b
    and a
    jr z, .go
.adv:
    ld a, l
    add a, 120
    ld l, a
    ld a, h
    adc a, 0
    ld h, a
    ld a, e
    add a, $c0
    ld e, a
    ld a, d
    adc a, 0
    ld d, a
    dec b
    jr nz, .adv
.go:
    ld b, 6
.r:
    ld c, 20
.c:
    ld a, [hl+]
    ld [de], a
    inc de
    dec c
    jr nz, .c
    ld a, e
    add a, 12
    ld e, a
    ld a, d
    adc a, 0
    ld d, a
    dec b
    jr nz, .r
    ret

; pokered ReadJoypad: select d-pad, read twice; select buttons, read six times
read_joypad:
    ld a, $20
    ldh [$00], a
    ldh a, [$00]
    ldh a, [$00]
    cpl
    and $0f
    swap a
    ld b, a
    ld a, $10
    ldh [$00], a
    ldh a, [$00]
    ldh a, [$00]
    ldh a, [$00]
    ldh a, [$00]
    ldh a, [$00]
    ldh a, [$00]
    cpl
    and $0f
    or b
    ld b, a
    ld a, $30
    ldh [$00], a
    ldh a, [hJoyHeld]
    ldh [hJoyLast], a
    ld c, a
    ld a, b
    ldh [hJoyHeld], a
    xor c
    and b
    ldh [hJoyPressed], a
    ret

dma_routine:
    db $e0, $46, $3e, $28, $3d, $20, $fd, $c9

text_data:
    db "HELLO THERE!", 0, 0, 0, 0
    db "A WILD MON!", 0, 0, 0, 0, 0
    db "GOT AN ITEM.", 0, 0, 0, 0
    db "THE GYM ....", 0, 0, 0, 0

; ---------------------------------------------------------------- bank 2: sound engine
section 2
org $4000
; 4 channels x 8 bytes at wSound: [timer, ptr_lo, ptr_hi(unused), vol, env, freq_lo, freq_hi, duty]
sound_update:
    ld hl, wSound
    ld c, $10
    ld b, 4
.ch:
    dec [hl]
    jr nz, .hold
    ; next note from the song table (indexed by the channel's note pointer)
    push hl
    inc hl
    ld a, [hl]
    inc a
    and $3f
    ld [hl+], a
    push bc
    ld e, a
    ld d, 0
    ld hl, song
    add hl, de
    add hl, de
    ld a, [hl+]
    ld e, a
    ld a, [hl]
    ld d, a
    pop bc
    pop hl
    ld a, e
    and $1f
    inc a
    ld [hl], a
    ; frequency registers (sound is not emulated: writes are ignored, like PyBoy without sound)
    ld a, c
    add a, 3
    push bc
    ld c, a
    ld a, d
    ld [c], a
    inc c
    ld a, e
    or $80
    ld [c], a
    pop bc
.hold:
    ; volume envelope step
    push hl
    inc hl
    inc hl
    inc hl
    ld a, [hl]
    and a
    jr z, .nov
    dec a
    ld [hl], a
.nov:
    pop hl
    ld a, l
    add a, 8
    ld l, a
    ld a, c
    add a, 5
    ld c, a
    dec b
    jr nz, .ch
    ld a, $77
    ldh [$24], a
    ldh a, [$25]
    or $ff
    ldh [$25], a
    ret

song:
    dw $0412, $0734, $0356, $0578, $069a, $03bc, $07de, $05f0
    dw $0421, $0743, $0365, $0587, $06a9, $03cb, $07ed, $050f
    dw $0412, $0734, $0356, $0578, $069a, $03bc, $07de, $05f0
    dw $0421, $0743, $0365, $0587, $06a9, $03cb, $07ed, $050f
    dw $0412, $0734, $0356, $0578, $069a, $03bc, $07de, $05f0
    dw $0421, $0743, $0365, $0587, $06a9, $03cb, $07ed, $050f
    dw $0412, $0734, $0356, $0578, $069a, $03bc, $07de, $05f0
    dw $0421, $0743, $0365, $0587, $06a9, $03cb, $07ed, $050f
    dw $0412, $0734

; ---------------------------------------------------------------- bank 3: battle engine
section 3
org $4000
battle_step:
    ld a, [wBattleTurn]
    and a
    jr nz, .turn
    ; battle start: decompress the enemy sprite into SRAM (pokered sSpriteBuffer)
    ld a, $0a
    ld [$0000], a
    xor a
    ld [$4000], a
    ld hl, $a000
    ld bc, 392
    ld e, $3c
.dec:
    ld a, e
    rlca
    xor c
    ld e, a
    ld [hl+], a
    dec bc
    ld a, b
    or c
    jr nz, .dec
    ; read it back (checksum into wMathR)
    ld hl, $a000
    ld b, 196
    xor a
.sum:
    add a, [hl]
    inc hl
    add a, [hl]
    inc hl
    dec b
    jr nz, .sum
    ld [wMathR], a
    xor a
    ld [$0000], a
    ld a, 1
    ld [wBattleTurn], a
    ret
.turn:
    ; every 8 frames one attack: damage = ((2*L/5+2) * P * A / D) / 50 + 2
    ldh a, [hFrameCounter]
    and 7
    ret nz
    call random
    and $1f
    add a, 20
    ld [wMathA], a
    xor a
    ld [wMathA + 1], a
    ld a, 40
    ld [wMathB], a
    call multiply16
    ld a, [wMathR]
    ld [wMathA], a
    ld a, [wMathR + 1]
    ld [wMathA + 1], a
    ld a, 35
    ld [wMathB], a
    call divide16
    ld a, [wMathR]
    srl a
    srl a
    srl a
    add a, 2
    ld b, a
    ld a, [wBattleTurn]
    and 1
    jr z, .enemy
    ld a, [wBattleEnemyHP]
    sub b
    jr nc, .e1
    xor a
.e1:
    ld [wBattleEnemyHP], a
    jr .hpbar
.enemy:
    ld a, [wBattleHP]
    sub b
    jr nc, .e2
    xor a
.e2:
    ld [wBattleHP], a
.hpbar:
    ; draw both HP bars into the tile map (rows 2 and 9)
    ld hl, wTileMap + 20 * 2 + 10
    ld a, [wBattleEnemyHP]
    call draw_bar
    ld hl, wTileMap + 20 * 9 + 2
    ld a, [wBattleHP]
    call draw_bar
    ld a, [wBattleTurn]
    inc a
    ld [wBattleTurn], a
    ld a, [wBattleEnemyHP]
    and a
    jr z, .end
    ld a, [wBattleHP]
    and a
    jr z, .end
    ld a, [wBattleTurn]
    cp 24
    ret c
.end:
    xor a
    ldh [hBattle], a
    ld a, 1
    ld [wMoved], a
    ret

; a = hp (0..63) -> 8 tiles of bar at hl
draw_bar:
    ld c, 8
.b:
    cp 8
    jr c, .partial
    sub 8
    ld [hl], $3f
    inc hl
    dec c
    jr nz, .b
    ret
.partial:
    ld b, a
.p:
    ld a, b
    add a, $30
    ld [hl+], a
    ld b, 0
    dec c
    jr nz, .p
    ret

; wMathR (16) = wMathA (16) * wMathB (8), shift-and-add
multiply16:
    ld hl, 0
    ld a, [wMathA]
    ld e, a
    ld a, [wMathA + 1]
    ld d, a
    ld a, [wMathB]
    ld b, 8
.m:
    srl a
    jr nc, .nadd
    add hl, de
.nadd:
    sla e
    rl d
    dec b
    jr nz, .m
    ld a, l
    ld [wMathR], a
    ld a, h
    ld [wMathR + 1], a
    ret

; wMathR (16) = wMathA (16) / wMathB (8), bit-serial long division
divide16:
    ld a, [wMathA]
    ld l, a
    ld a, [wMathA + 1]
    ld h, a
    ld a, [wMathB]
    ld c, a
    xor a
    ld b, 16
.d:
    add hl, hl
    rla
    jr c, .sub
    cp c
    jr c, .nsub
.sub:
    sub c
    inc l
.nsub:
    dec b
    jr nz, .d
    ld a, l
    ld [wMathR], a
    ld a, h
    ld [wMathR + 1], a
    ret
"""


# Routines the banked variant relocates out of the home bank (pokered keeps its overworld engine,
# map scripts and text in many switchable banks and reaches them through Bankswitch every frame).
# prepare_oam / put_tile stay home: the VBlank handler calls them with any bank mapped.
BANKED_ROUTINES = ("update_npcs", "update_sprites", "draw_map_view", "text_engine", "menu_logic")
FIRST_OW_BANK = 4


def _routines(src: str) -> dict[str, str]:
    """Global-label spans of the home bank (label line up to the next global label)."""
    home = src[:src.index("section 2")]
    marks = [(m.start(), m.group(1)) for m in re.finditer(r"^([A-Za-z_]\w*):", home, re.M)]
    marks.append((len(home), None))
    return {name: home[a:b] for (a, name), (b, _) in zip(marks, marks[1:])}


def banked_source(n_banks: int) -> str:
    """`pkbench` re-laid-out for an n_banks cartridge (64 = 1 MiB, pokemon_red.gb's size): the
    overworld engine (NPCs, sprite state, map view, text, menu) plus a per-bank map script lives in
    banks FIRST_OW_BANK..n_banks-1, one copy per bank; every frame the main loop picks the bank of
    the player's 4x4-metatile region, (x/4 + 16*(y/4)) mod (n_banks - 4), and reaches its engine
    through a Bankswitch trampoline (save hROMBank, switch, call $4000, restore), so envs in
    different regions run code from different banks and most executed code sits outside the six
    banks K1 stages in LDS."""
    nb = n_banks - FIRST_OW_BANK
    spans = _routines(SRC)
    home = SRC[:SRC.index("section 2")]
    for name in BANKED_ROUTINES:
        home = home.replace(spans[name], "")
    main_old = """    call update_npcs
    call update_sprites
    ld a, [wMoved]
    and a
    call nz, draw_map_view
    call text_engine
    call menu_logic
"""
    main_new = f"""    ; region -> bank: 4 + (x/4 + 16*(y/4)) mod {nb}
    ld a, [wPlayerX]
    rrca
    rrca
    and $0f
    ld b, a
    ld a, [wPlayerY]
    add a, a
    add a, a
    and $f0
    or b
.mod:
    cp {nb}
    jr c, .inr
    sub {nb}
    jr .mod
.inr:
    add a, {FIRST_OW_BANK}
    call farcall_ow
"""
    assert main_old in home
    home = home.replace(main_old, main_new)
    home = home.replace("farcall_battle:", """farcall_ow:
    ; pokered Bankswitch into the region's overworld bank: the engine entry is at $4000
    ld b, a
    ldh a, [hROMBank]
    push af
    ld a, b
    ldh [hROMBank], a
    ld [$2000], a
    call $4000
    pop af
    ldh [hROMBank], a
    ld [$2000], a
    ret

farcall_battle:""")
    out = [home, SRC[SRC.index("section 2"):]]
    for b in range(FIRST_OW_BANK, n_banks):
        body = "".join(spans[name] for name in BANKED_ROUTINES)
        for name in BANKED_ROUTINES:
            body = re.sub(rf"\b{name}\b", f"{name}_b{b}", body)
        # a map script per bank: fold 16 bytes of this bank's table (chosen by the frame counter)
        # into wMathR — data reads from the switched bank, like pokered's map headers and text
        table = ", ".join(f"${(b * 37 + k * 11) & 0xFF:02x}" for k in range(32))
        out.append(f"""
section {b}
org $4000
ow_entry_b{b}:
    call update_npcs_b{b}
    call update_sprites_b{b}
    ld a, [wMoved]
    and a
    call nz, draw_map_view_b{b}
    call text_engine_b{b}
    call menu_logic_b{b}
    ldh a, [hFrameCounter]
    and $0f
    ld hl, script_table_b{b}
    add a, l
    ld l, a
    ld a, h
    adc a, 0
    ld h, a
    ld a, [wMathR]
    ld c, a
    ld b, 16
.s:
    ld a, [hl+]
    xor c
    rlca
    ld c, a
    dec b
    jr nz, .s
    ld a, c
    ld [wMathR], a
    ret
{body}
script_table_b{b}:
    db {table}
""")
    return "".join(out)


def game_rom(banks: int = 4) -> bytes:
    """pkbench: banks=4 is the benchmark ROM of round 1 (every bank fits the LDS staging);
    banks=64 is the 1 MiB layout with the overworld engine spread over 60 switchable banks."""
    if banks == 4:
        return build_rom(SRC, n_banks=4, title="PKBENCH")
    if banks < 8 or banks & (banks - 1) or banks > 128:
        raise ValueError("banks must be 4 or a power of two in [8, 128]")
    return build_rom(banked_source(banks), n_banks=banks, title=f"PKBENCH{banks}")
