"""Projects the unit cube with an orthographic and a perspective camera."""
import bpy
from blendtorch import btb

btargs, remainder = btb.parse_blendtorch_args()
cube = bpy.data.objects['Cube']
ortho = btb.Camera(bpy.data.objects['CamOrtho'])
proj = btb.Camera(bpy.data.objects['CamProj'])
xyz = btb.utils.world_coordinates(cube)
proj_ndc, proj_z = proj.world_to_ndc(xyz, return_depth=True)
ortho_ndc, ortho_z = ortho.world_to_ndc(xyz, return_depth=True)
pub = btb.DataPublisher(btargs.btsockets['DATA'], btargs.btid, lingerms=5000)
pub.publish(ortho_xy=ortho.ndc_to_pixel(ortho_ndc, origin='upper-left'), ortho_z=ortho_z,
            proj_xy=proj.ndc_to_pixel(proj_ndc, origin='upper-left'), proj_z=proj_z,
            obj_px=proj.object_to_pixel(cube), bbox_px=proj.bbox_object_to_pixel(cube))
